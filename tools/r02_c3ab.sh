#!/bin/bash
# GPU box: block-kernel parity tests, then C3 A/B of two library builds.
set -o pipefail
OUT=gpurun_out/c3ab; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "block or config3 or 64x64 or big or 50x50 or odd or f64 or param_points" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_core.sh "build_ab/lib_c3base.so build_ab/lib_c3new.so" --config 3 --multi-step 0 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
