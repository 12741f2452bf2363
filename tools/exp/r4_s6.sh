# Round 4, session 6: committed GCM changes (8 lanes for ragged / extra-byte
# one-key batches) + the one-record kernel: GPU suite, single-record latency,
# bench lines with parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s6
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -2 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest 1500 python -u -m pytest tests/ -q -m gpu -x -rf --timeout 300 --timeout-method thread
step latency 300 python tools/latency_bench.py
for c in config2 configG config4 config5 config3; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline
done
