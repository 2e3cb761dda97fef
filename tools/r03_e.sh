#!/bin/bash
# GPU box: C5 touched-slot fractions, the 8-rank C4 rehearsal (exchange volume with
# adaptive record capacity), the actor pins at several env counts.
set -o pipefail
OUT=gpurun_out/${1:-e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 bash tools/c5_profile.sh r03_e/c5prof > "$OUT/c5prof.out" 2>&1 || { echo "c5 profile failed"; tail -20 "$OUT/c5prof.out"; exit 1; }
grep LSTAMP "$OUT/c5prof.out" | tail -4
timeout -k 10 300 python3 tools/c5_touched.py 512 4096 > "$OUT/c5_touched.log" 2>&1 || { echo "touched failed"; tail -20 "$OUT/c5_touched.log"; exit 1; }
grep -v "^{" "$OUT/c5_touched.log" | tail -14
timeout -k 10 600 bash tools/rehearse.sh r03_e/rehearse_c4 8 --config 4 --steps 20 --warmup 40 --repeats 2 > "$OUT/rehearse_c4.out" 2>&1 || { echo "rehearse failed"; tail -20 "$OUT/rehearse_c4.out"; exit 1; }
tail -1 "$OUT/rehearse_c4.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['table_sync']), d['value'])"
timeout -k 10 600 bash tools/rehearse.sh r03_e/rehearse_c5 2 --config 5 --steps 3 --warmup 2 --repeats 1 > "$OUT/rehearse_c5.out" 2>&1 || { echo "rehearse c5 failed"; tail -20 "$OUT/rehearse_c5.out"; exit 1; }
tail -1 "$OUT/rehearse_c5.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['table_sync']), d['value'])"
timeout -k 10 900 bash tools/actor_pin.sh r03_e/actor_pin 10 512 4096 > "$OUT/actor_pin.out" 2>&1 || { echo "actor pin failed"; tail -20 "$OUT/actor_pin.out"; exit 1; }
cat "$OUT/actor_pin.out"

timeout -k 10 600 bash tools/traffic.sh gpurun_out/r03_e/traffic_c5 --config 5 > "$OUT/traffic_c5.out" 2>&1 || { echo "traffic c5 failed"; tail -20 "$OUT/traffic_c5.out"; exit 1; }
tail -30 "$OUT/traffic_c5.out"
timeout -k 10 900 bash tools/pmc_kern.sh gpurun_out/r03_e/pmc_c2 "" > "$OUT/pmc_c2.out" 2>&1 || { echo "pmc c2 failed"; tail -20 "$OUT/pmc_c2.out"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r03_e/pmc_c2/k1 core_group > "$OUT/pmc_c2_summary.txt"; cat "$OUT/pmc_c2_summary.txt"
timeout -k 10 600 bash tools/traffic.sh gpurun_out/r03_e/traffic_c2 > "$OUT/traffic_c2.out" 2>&1 || { echo "traffic c2 failed"; tail -20 "$OUT/traffic_c2.out"; exit 1; }
tail -14 "$OUT/traffic_c2.out"
