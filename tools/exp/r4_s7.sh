# Round 4, session 7: the table-free engine for every GCM batch (bs16 mode
# suite), the whole GPU suite, single-record latency + kernel trace, bs16
# bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s7
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
step bs16 1200 python -u -m pytest tests/test_bs16_total.py -v -m gpu -x -rf --timeout 300 --timeout-method thread
step pytest 1500 python -u -m pytest tests/ -q -m gpu -x -rf --timeout 300 --timeout-method thread
step latency 300 python tools/latency_bench.py
step latency_trace 300 rocprofv3 --kernel-trace --stats -d $O/lat_prof -o lat -- python tools/latency_bench.py
for c in config2 configG config4 config5; do
  step bs16_$c 300 env BSSL_AMD_GCM_MODE=bs16 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline
done
