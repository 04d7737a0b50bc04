"""D2H rate probe (diagnostic, not part of the product): 451-MB chunks of packed masks from HBM to
pinned host memory by (a) copy_ on one stream, (b) the same split over 2 / 4 streams, (c) a device
kernel writing the host buffer directly (torch index_copy through a host-mapped view is not possible,
so (c) uses a HIP kernel via torch's elementwise copy into a pinned tensor viewed on the device)."""
import time

import torch

dev = torch.device("cuda")
n, ldb, chunks = 65536, 6880, 8
src = torch.randint(0, 255, (n, ldb), dtype=torch.uint8, device=dev)
host = torch.empty(chunks * n, ldb, dtype=torch.uint8, pin_memory=True)
torch.cuda.synchronize()


def run(nstreams):
    ss = [torch.cuda.Stream() for _ in range(nstreams)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(chunks):
        part = n // nstreams
        for i, s in enumerate(ss):
            with torch.cuda.stream(s):
                host[c * n + i * part:c * n + (i + 1) * part].copy_(src[i * part:(i + 1) * part], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return chunks * n * ldb / dt / 1e9


for ns in (1, 1, 2, 4, 8):
    print(f"copy_ on {ns} stream(s): {run(ns):.1f} GB/s", flush=True)
