# Round 4, session 5: quad-split E_K(J0) at unit start, 8 lanes per record for
# every uniform one-key batch; variants: 8 lanes for ragged batches (l8r),
# next unit claimed two iterations early (ce), 16 lanes above 4 KiB (l16u).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s5
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
B=$PWD/boringssl_amd/csrc/build
step par_l8r_4 300 env BSSL_AMD_LIB=$B/ab_l8r/libbssl_amd.so python bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline
step par_ce_G 300 env BSSL_AMD_LIB=$B/ab_ce/libbssl_amd.so python bench.py --config configG --steps 2 --warmup 1 --no-cpu-baseline
step par_ce_2 300 env BSSL_AMD_LIB=$B/ab_ce/libbssl_amd.so python bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline
step par_ce_4 300 env BSSL_AMD_LIB=$B/ab_ce/libbssl_amd.so python bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline
SPECS="configG:ab_ce,ab_r3 config2:ab_ce,ab_l16u,ab_r3 config4:ab_l8r,ab_ce,ab_r3 config5:ab_r3" REPS="1 2" step ab 1200 bash tools/exp/ab_session.sh
cat $O/ab.log
