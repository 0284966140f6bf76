"""RCCL probe (no swarm_amd code): a 1-rank "nccl" process group on cuda:0, async byte
all-to-alls between device buffers, each checked with torch.equal. Bisects the fault seen in
the 1-rank forced-exchange C5 rounds step at 1B records (1.65 GB rounds).
  python3 tools/rccl_probe.py sizes <MB> [<MB> ...]       one all_to_all_single per size
  python3 tools/rccl_probe.py offsets <MB> <GB> [<GB> ...] one message of MB at each send offset
  python3 tools/rccl_probe.py list <MB> [<MB> ...]        list all_to_all (grouped send/recv)
  python3 tools/rccl_probe.py chunked <MB> <chunk MB>     swarm_amd's chunked all_to_all_bytes
  python3 tools/rccl_probe.py detail <MB>                 what arrived: fill/zero/shifted bytes, guards
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
    elif mode == "detail":
        # What arrives when the message is wrong: recv sits in the middle of one guarded
        # allocation pre-filled with 0xAB, so bytes RCCL never wrote keep the fill, and a write
        # outside recv shows up in the guards. Mismatches are classified: untouched (fill),
        # zero, a copy of send from another offset (shift found from the first mismatch), other.
        mb = int(sys.argv[2])
        n = mb << 20
        guard = 64 << 20
        send = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        send[send == 0xAB] = 0x5A  # the fill value never occurs in send
        big = torch.full((n + 2 * guard,), 0xAB, dtype=torch.uint8, device="cuda")
        recv = big[guard:guard + n]
        t0 = time.perf_counter()
        w = dist.all_to_all_single(recv, send, output_split_sizes=[n], input_split_sizes=[n], async_op=True)
        w.wait()
        torch.cuda.synchronize()
        print("detail %d MB: %.3f s" % (mb, time.perf_counter() - t0), flush=True)
        gl, gr = big[:guard], big[guard + n:]
        print("guard before: %d bytes changed; guard after: %d bytes changed" %
              (int((gl != 0xAB).sum()), int((gr != 0xAB).sum())), flush=True)
        bad = (recv != send).nonzero().flatten()
        print("mismatched bytes: %d of %d" % (bad.numel(), n), flush=True)
        if bad.numel():
            first, last = int(bad[0]), int(bad[-1])
            rb = recv[bad]
            print("first mismatch at %d (%.4f GiB), last at %d (%.4f GiB)" %
                  (first, first / (1 << 30), last, last / (1 << 30)), flush=True)
            print("untouched (0xAB fill): %d, zero: %d, other: %d" %
                  (int((rb == 0xAB).sum()), int((rb == 0).sum()), int(((rb != 0xAB) & (rb != 0)).sum())), flush=True)
            # contiguous mismatch runs (up to 8 listed)
            if bad.numel() > 1:
                brk = ((bad[1:] - bad[:-1]) != 1).nonzero().flatten()
                starts = [first] + [int(bad[int(i) + 1]) for i in brk[:7]]
                ends = [int(bad[int(i)]) for i in brk[:8]] + ([last] if brk.numel() < 8 else [])
                print("mismatch runs (first 8):", list(zip(starts, ends)), "of", int(brk.numel()) + 1, flush=True)
            win = recv[first:first + 32].cpu().tolist()
            print("recv at first mismatch:", bytes(win).hex(), flush=True)
            print("send at first mismatch:", bytes(send[first:first + 32].cpu().tolist()).hex(), flush=True)
            # is it a copy of send from another offset? (candidate shifts: powers of two)
            pat = recv[first:first + 16]
            found = []
            for sft in [0] + [sg * (1 << k) for k in range(20, 33) for sg in (1, -1)] + [-first]:
                o = first + sft
                if 0 <= o <= n - 16 and torch.equal(send[o:o + 16], pat):
                    found.append("%d (shift %+d)" % (o, sft))
            print("first mismatch's 16 bytes found in send at:", found or "none of the candidate shifts",
                  flush=True)
        del send, big, recv  # (informational: exits 0 either way)
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
