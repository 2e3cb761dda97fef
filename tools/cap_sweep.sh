set -o pipefail
export TMPDIR=/tmp
for lg in 17 19 21 23; do
  v=$(timeout -k 10 120 python3 bench.py --no-cpu --config 4 --steps 100 --warmup 5 --log2-table $lg 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['step_ms_events']*1000,1), 'us', round(d['ms_per_step']*1000,1), d['tables'])") || exit 1
  echo "log2 $lg: $v"
done
