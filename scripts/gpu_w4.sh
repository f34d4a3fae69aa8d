#!/bin/bash
# A/B: dual launches forced to 4 waves per SIMD (side build _C_w4.so, DDL_DUAL_WAVES=4)
set -u
cd "$(dirname "$0")/.."
SO_B=_C_w4.so SKIP_TESTS=1 bash scripts/gpu_so_ab.sh 3
