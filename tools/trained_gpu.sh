#!/bin/bash
# GPU box: the ffm_trained_core parity tests (learner goldens, drop-in class, batched).
set -o pipefail
mkdir -p gpurun_out/trained
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py tests/test_gpu_dropin_learn.py -x -v -k "trained" --timeout 600 --timeout-method thread > gpurun_out/trained/pytest.log 2>&1 || { echo "failed"; tail -40 gpurun_out/trained/pytest.log; exit 1; }
tail -3 gpurun_out/trained/pytest.log
