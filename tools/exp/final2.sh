# Round-3 re-validation of HEAD on one GPU (smoke, GPU suite, default bench,
# config G bench + rocprofv3 stats and PMC passes).  Each step has its own
# limit; a fault ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/final2
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest 1200 python -u -m pytest tests/ -v -m gpu -rf --timeout 300 --timeout-method thread
step bench 600 python bench.py
step bench_configG 600 python bench.py --config configG
O=$O/prof CONFIGS="configG" PASSES="stats pmc" bash tools/profile.sh
