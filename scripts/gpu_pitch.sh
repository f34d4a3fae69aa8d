#!/bin/bash
# conv1 kernels' LDS pitch (48 / 37, conflict-free) vs 32: kernel tests, then same-box A/B of builds
set -u
cd "$(dirname "$0")/.."
TESTS="tests/test_hip_kernels.py" SO_B=_C_p32.so bash scripts/gpu_so_ab.sh 3
