#!/bin/bash
# GPU box: Philox parity (all kernels use wave_reset_env), then C2 A/B of placement variants.
set -o pipefail
OUT=gpurun_out/rank2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "philox" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_core.sh "build_ab/lib_g_base.so build_ab/lib_g_rank2.so build_ab/lib_g_rank2twice.so" --multi-step 0 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
