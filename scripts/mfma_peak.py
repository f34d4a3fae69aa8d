"""Measure the sustained fp32 MFMA rate (TFLOP/s) and implied clock on this GPU."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.ops import native
ext = native.ops()
iters = 20000
for kind, blocks in [(k, b) for k in (0, 1) for b in (1024, 2048, 4096, 8192)]:
    out = torch.zeros(blocks * 64, device="cuda")
    ext.mfma_peak(out, blocks, 10, kind)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    ext.mfma_peak(out, blocks, iters, kind)
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en)
    flop = blocks * 2 * iters * 32 * 32 * 2 * 2
    tf = flop / ms / 1e9
    # 1024 SIMDs x 64 FLOP/clk
    print(f"{('32x32x2', '16x16x4')[kind]} waves={blocks:5d}  {ms:8.3f} ms  {tf:7.1f} TFLOP/s  implied clock {tf * 1e12 / (1024 * 64) / 1e9:5.2f} GHz", flush=True)

# GEMM structure without memory traffic (32x32 one-wave tiles, BK=32), conv2-fwd shape
out = torch.zeros(4096, device="cuda")
for M, N, K, s in [(19600, 64, 800, 4), (19600, 64, 800, 1), (6400, 128, 1600, 4), (1600, 128, 6400, 16)]:
    slab = torch.zeros(max(1, s) * ((M + 31) // 32) * ((N + 31) // 32) * 1024 * 4, device="cuda")
    ext.gemm_nomem(out, slab, M, N, K, s)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20):
        ext.gemm_nomem(out, slab, M, N, K, s)
    en.record()
    torch.cuda.synchronize()
    us = 1e3 * st.elapsed_time(en) / 20
    print(f"nomem gemm M={M} N={N} K={K} s={s}: {us:7.1f} us  {2 * M * N * K / us / 1e6:6.1f} TF", flush=True)
