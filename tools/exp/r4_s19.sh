# Round 4, session 19: 4 lanes per record for short uniform records (ab_l4):
# config G digest check and A/B against main.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s19
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
step par_l4_G 200 env BSSL_AMD_LIB=$B/ab_l4/libbssl_amd.so python bench.py --config configG --steps 2 --warmup 1 --no-cpu-baseline
SPECS="configG:ab_l4" REPS="1 2 3" STEPS=20 step ab 400 bash tools/exp/ab_session.sh
cat $O/ab.log
