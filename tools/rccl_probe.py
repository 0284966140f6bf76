"""RCCL probe (no swarm_amd code): a 1-rank "nccl" process group on cuda:0, async byte
all-to-alls between device buffers, each checked with torch.equal. Bisects the fault seen in
the 1-rank forced-exchange C5 rounds step at 1B records (1.65 GB rounds).
  python3 tools/rccl_probe.py sizes <MB> [<MB> ...]       one all_to_all_single per size
  python3 tools/rccl_probe.py offsets <MB> <GB> [<GB> ...] one message of MB at each send offset
  python3 tools/rccl_probe.py list <MB> [<MB> ...]        list all_to_all (grouped send/recv)
  python3 tools/rccl_probe.py chunked <MB> <chunk MB>     swarm_amd's chunked all_to_all_bytes
Exits 1 at the first mismatch.
Round 4 result (5 queued messages): 64..512 MB equal, 1800 MB NOT equal."""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist


def check(tag, recv, ref, t0):
    torch.cuda.synchronize()
    ok = torch.equal(recv, ref)
    print("%s: equal %s, %.3f s" % (tag, ok, time.perf_counter() - t0), flush=True)
    return ok


def main():
    mode = sys.argv[1]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % port)
    if mode in ("sizes", "list"):
        for mb in [int(x) for x in sys.argv[2:]]:
            n = mb << 20
            send = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
            recv = torch.empty(n, dtype=torch.uint8, device="cuda")
            t0 = time.perf_counter()
            if mode == "sizes":
                w = dist.all_to_all_single(recv, send, output_split_sizes=[n], input_split_sizes=[n], async_op=True)
            else:
                w = dist.all_to_all([recv], [send], async_op=True)
            w.wait()
            ok = check("%s %d MB" % (mode, mb), recv, send, t0)
            del send, recv
            if not ok:
                sys.exit(1)
    elif mode == "offsets":
        mb = int(sys.argv[2])
        n = mb << 20
        offs = [int(float(x) * (1 << 30)) for x in sys.argv[3:]]
        send = torch.randint(0, 256, (max(offs) + n,), dtype=torch.uint8, device="cuda")
        for o in offs:
            recv = torch.empty(n, dtype=torch.uint8, device="cuda")
            t0 = time.perf_counter()
            w = dist.all_to_all_single(recv, send[o:o + n], output_split_sizes=[n], input_split_sizes=[n],
                                       async_op=True)
            w.wait()
            if not check("offset %.2f GB, %d MB" % (o / (1 << 30), mb), recv, send[o:o + n], t0):
                sys.exit(1)
    elif mode == "chunked":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from swarm_amd import distributed as D
        mb, cmb = int(sys.argv[2]), int(sys.argv[3])
        D.A2A_CHUNK = cmb << 20
        n = mb << 20
        send = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        recv = torch.empty(n, dtype=torch.uint8, device="cuda")
        t0 = time.perf_counter()
        w = D.all_to_all_bytes(recv, send, [n], [n], async_op=True)
        w.wait()
        if not check("chunked %d MB in %d MB pieces" % (mb, cmb), recv, send, t0):
            sys.exit(1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
