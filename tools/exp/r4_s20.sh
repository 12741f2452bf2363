# Round 4, session 20: 4 lanes per record for uniform batches of short
# records (main) -- GPU suite, bench lines; A/B of 4 lanes for every one-key
# batch (ab_l4all) on configs 4 and 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s20
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
B=$PWD/boringssl_amd/csrc/build
echo "[$(date +%T)] pytest" | tee -a $O/steps.log
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc" | tee -a $O/steps.log
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for c in configG config2 config4; do step bench_$c 200 python bench.py --config $c --no-cpu-baseline; done
step par_l4all_4 200 env BSSL_AMD_LIB=$B/ab_l4all/libbssl_amd.so python bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline
SPECS="config4:ab_l4all config2:ab_l4all" REPS="1 2" STEPS=10 step ab 600 bash tools/exp/ab_session.sh
cat $O/ab.log
