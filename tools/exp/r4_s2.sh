# Round 4, session 2: the fused GCM record start (no prologue kernel) and the
# trimmed sources -- smoke, the whole GPU suite, then same-box A/B against the
# round-3 gcm.hip (boringssl_amd/csrc/build/ab_r3).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s2
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest 1500 python -u -m pytest tests/ -v -m gpu -x -rf --timeout 300 --timeout-method thread
SPECS="configG:ab_r3 config2:ab_r3 config4:ab_r3 config5:ab_r3" REPS="1 2" step ab 900 bash tools/exp/ab_session.sh
cat $O/ab.log
