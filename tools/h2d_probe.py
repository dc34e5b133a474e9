#!/usr/bin/env python3
"""Host-to-device copy rate of a pageable 1.47 GB payload (bench.py's host-CSR
leg at 256^3: int32 indptr/indices + fp64 data), one copy against K chunks on
K streams from K host threads.
    python tools/h2d_probe.py [--fresh] [K ...]   (--fresh: a new host array per copy)"""
import sys, threading, time
import numpy as np, torch

nbytes = 1_471_676_420
src = np.ones(nbytes // 8, dtype=np.float64)
dev = torch.empty(src.size, dtype=torch.float64, device="cuda")
FRESH = "--fresh" in sys.argv
ks = [int(v) for v in sys.argv[1:] if v != "--fresh"] or [1, 2, 4, 8]
for rep in range(2):
    for k in ks:
        streams = [torch.cuda.Stream() for _ in range(k)]
        edges = np.linspace(0, src.size, k + 1).astype(np.int64)
        def work(q):
            with torch.cuda.stream(streams[q]):
                dev[edges[q]:edges[q + 1]].copy_(torch.from_numpy(src[edges[q]:edges[q + 1]]), non_blocking=False)
            streams[q].synchronize()
        if FRESH:                     # a new host payload each time: its pages never copied before
            src = np.ones(nbytes // 8, dtype=np.float64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = [threading.Thread(target=work, args=(q,)) for q in range(k)]
        for t in ts: t.start()
        for t in ts: t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {rep} K={k}: {dt * 1e3:7.1f} ms  {nbytes / dt / 1e9:6.1f} GB/s", flush=True)
