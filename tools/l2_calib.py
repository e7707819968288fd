#!/usr/bin/env python3
"""Calibration pass for the L2 request counters (tools/gpu.sh profile): a device-to-device copy of
known bytes (256 MiB read + 256 MiB written, 5 times) under the same `--pmc TCC_REQ_sum TCC_HIT_sum
TCC_MISS_sum` pass as the bench, so tools/limiters.py can turn TCC_REQ into bytes per request for
streaming 16-byte-per-lane accesses (MI355X_MICROARCH.md: the memory-side counters tally 128-B
requests at 64 B; the request size is measured here, not assumed)."""
import torch

n = 1 << 26  # f32 elements: 256 MiB
x = torch.ones(n, dtype=torch.float32, device="cuda")
y = torch.empty_like(x)
for _ in range(5):
    y.copy_(x)
torch.cuda.synchronize()
print("copied", 5 * 2 * x.numel() * 4, "bytes (read + written) in 5 launches")
