"""PCIe host->device copy rate on this box: pinned sources, 1 / 2 / 4 concurrent copy streams,
chunk sizes around one 64K x 324 B batch.  Used to set the PCIe bound of the headline."""
import json
import sys

import torch

dev = torch.device("cuda", 0)
res = {}
for chunk_mb in (4, 21, 64):
    nb = chunk_mb << 20
    for nstreams in (1, 2, 4):
        srcs = [torch.empty(nb, dtype=torch.uint8).pin_memory() for _ in range(nstreams)]
        dsts = [torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(nstreams)]
        streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
        reps = max(4, 512 // chunk_mb // nstreams)
        for _ in range(2):
            for s, a, b in zip(streams, srcs, dsts):
                with torch.cuda.stream(s):
                    b.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        for _ in range(reps):
            for s, a, b in zip(streams, srcs, dsts):
                with torch.cuda.stream(s):
                    b.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[f"{chunk_mb}MB_x{nstreams}"] = reps * nstreams * nb / dt / 1e9
json.dump(res, sys.stdout, indent=1)
print()
