# Headline value against timed/warmup solve counts (pairs "steps warmup"), two passes.
set -o pipefail
for r in 1 2; do
for cfg in "20 5" "50 20" "200 50" "20 200"; do
  set -- $cfg
  v=$(timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-secondary | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(round(j['value']/1e9,4), round(j['ms_per_step'],4))") || exit 1
  echo "steps=$1 warmup=$2 -> $v"
done
done
