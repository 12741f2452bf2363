# Round 4, session 4: split one-key / keyset GCM kernels, 8 lanes per record
# for short uniform records.  Full GPU suite on main, parity of the variants
# on the bench workloads, then same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s4
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
step par_pipe_G 300 env BSSL_AMD_LIB=$B/ab_pipe/libbssl_amd.so python bench.py --config configG --steps 2 --warmup 1 --no-cpu-baseline
step par_pipe_2 300 env BSSL_AMD_LIB=$B/ab_pipe/libbssl_amd.so python bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline
step par_l8all_2 300 env BSSL_AMD_LIB=$B/ab_l8all/libbssl_amd.so python bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline
SPECS="configG:ab_pipe,ab_l16,ab_r3 config2:ab_pipe,ab_l8all,ab_r3 config4:ab_pipe,ab_r3 config5:ab_r3" REPS="1 2" step ab 1200 bash tools/exp/ab_session.sh
cat $O/ab.log
