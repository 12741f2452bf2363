# Round-3 final evidence on one GPU: smoke, GPU suite, default bench, every
# config's bench with its digest check, rocprofv3 stats + PMC passes, and the
# 2-rank launcher rehearsal.  Each step has its own limit; a fault ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/final
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
for c in config3 config3x config4 config5 configS; do step bench_$c 600 python bench.py --config $c --no-cpu-baseline; done
step bench_config2_open 300 python bench.py --op open --no-cpu-baseline
step bench_config3_open 300 python bench.py --config config3 --op open --no-cpu-baseline
step rehearse2 600 env BSSL_AMD_REHEARSE_DEVICES=1 python bench.py --gpus 2 --no-cpu-baseline
O=$O/prof CONFIGS="config2 config3 config3x config4 config5 configS" PASSES="stats pmc" bash tools/profile.sh
