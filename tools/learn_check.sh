#!/bin/bash
# GPU box: learner GPU tests, then the actor-dynamics pin (tools/actor_pin.sh).
set -o pipefail
OUT=gpurun_out/learn_check; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py tests/test_gpu_dropin_learn.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/actor_pin.sh
