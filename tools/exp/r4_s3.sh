# Round 4, session 3: the next-unit pipeline (claim two iterations before the
# unit ends, next unit's loads before the record end) -- parity of the
# variant on the bench workloads, then same-box A/B against the fused build
# (main) and round 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s3
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
V=$PWD/boringssl_amd/csrc/build/ab_pipe/libbssl_amd.so
for c in configG config2 config4 config5; do
  step parity_pipe_$c 300 env BSSL_AMD_LIB=$V python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline
done
step tests_pipe 900 env BSSL_AMD_LIB=$V python -u -m pytest tests/test_gpu_parity.py tests/test_aead_api_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread
SPECS="configG:ab_pipe,ab_r3 config2:ab_pipe,ab_r3 config4:ab_pipe,ab_r3 config5:ab_pipe" REPS="1 2" step ab 900 bash tools/exp/ab_session.sh
cat $O/ab.log
