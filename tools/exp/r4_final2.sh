# Round-4 final evidence, second run on the last build (part 1): every config's bench line with
# its digest check (config 2 with the CPU baseline), open lines, the 2-rank
# rehearsal, and rocprofv3 kernel stats of the bench commands.  Part 2
# (r4_final_pmc.sh): the PMC passes.  The GPU suite, smoke and latency of the
# final build: r4_check.sh.  Each step has its own limit; the chain stops at
# the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4final2
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
step bench 600 python bench.py
for c in configG config3 config3x config4 config5 configS; do
  step bench_$c 300 python bench.py --config $c --no-cpu-baseline
done
step bench_config2_open 300 python bench.py --op open --no-cpu-baseline
step bench_config3_open 300 python bench.py --config config3 --op open --no-cpu-baseline
step rehearse2 300 env BSSL_AMD_REHEARSE_DEVICES=1 python bench.py --gpus 2 --no-cpu-baseline
step latency 200 python tools/latency_bench.py
step latency_2 200 python tools/latency_bench.py
step latency_c 120 tools/latency_c
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
O=$O/prof CONFIGS="config2 configG config3 config4 config5" PASSES="stats pmc" bash tools/profile.sh
