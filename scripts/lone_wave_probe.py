"""Per-wave rates with few waves on the chip (no contention): the raw MFMA chain (two
accumulator chains, register operands) and the engine's 32x32 BK 32 K loop without memory
traffic (register-only 'loads'), in us per 16 MFMAs (one K tile)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.ops import native  # noqa: E402

ext = native.ops()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return 1e3 * st.elapsed_time(en) / reps


iters = 20000
for blocks in (8, 64, 256, 1024):
    out = torch.zeros(blocks * 64, device="cuda")
    us = timed(lambda: ext.mfma_peak(out, blocks, iters))
    print(f"mfma chain  waves={blocks:5d}: {us / (iters * 2 / 16):.3f} us per 16 MFMAs "
          f"({us * 1e3 / (iters * 2):.1f} ns per MFMA)", flush=True)
out = torch.zeros(4096, device="cuda")
for M, N, K in [(32 * 26, 64, 19600), (32 * 8, 32, 19600)]:
    slab = torch.zeros(1024 * 4 * 64, device="cuda")
    us = timed(lambda: ext.gemm_nomem(out, slab, M, N, K, 1))
    tiles = (K + 31) // 32
    print(f"nomem K loop blocks={(M // 32) * (N // 32):4d} K tiles={tiles}: "
          f"{us / tiles:.3f} us per K tile", flush=True)
