# Round 4, session 16: nonce and short AD by value for single records, LDS-only
# barrier in the one-record GCM kernel -- smoke, GPU suite, single-record
# latency from C (tools/latency_c) and from Python (tools/latency_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s16
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
echo "[$(date +%T)] pytest" | tee -a $O/steps.log
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc" | tee -a $O/steps.log
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2 3; do
  step latency_c_$r 120 tools/latency_c
  step latency_py_$r 200 python tools/latency_bench.py
done
