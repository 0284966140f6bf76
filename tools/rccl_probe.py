"""RCCL probe (no swarm_amd code): a 1-rank "nccl" process group on cuda:0, async byte
all_to_all_single calls of growing size between device buffers, each checked with
torch.equal. Bisects a fault seen in the 1-rank forced-exchange C5 rounds step at 1B records
(1.65 GB rounds): does RCCL itself handle GB-sized self messages?
  python3 tools/rccl_probe.py [max_mb] [queued]"""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist


def main():
    max_mb = int(sys.argv[1]) if len(sys.argv) > 1 else 1800
    queued = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % port)
    mb = 64
    while mb <= max_mb:
        n = mb << 20
        send = torch.randint(0, 256, (n * queued + 7,), dtype=torch.uint8, device="cuda")
        recvs, works = [], []
        t0 = time.perf_counter()
        for q in range(queued):
            r = torch.empty(n, dtype=torch.uint8, device="cuda")
            w = dist.all_to_all_single(r, send[q * n:(q + 1) * n], output_split_sizes=[n], input_split_sizes=[n],
                                       async_op=True)
            recvs.append(r)
            works.append(w)
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        ok = all(torch.equal(recvs[q], send[q * n:(q + 1) * n]) for q in range(queued))
        print("size %d MB x %d queued: equal %s, %.3f s" % (mb, queued, ok, time.perf_counter() - t0), flush=True)
        if not ok:
            break
        del send, recvs, works
        mb *= 2 if mb < 1024 else 1
        if mb >= 1024:
            mb = max_mb if mb < max_mb else max_mb + 1
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
