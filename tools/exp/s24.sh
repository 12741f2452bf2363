set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/s24_tests.txt 2>&1 || { tail -30 gpurun_out/s24_tests.txt; exit 1; }
tail -2 gpurun_out/s24_tests.txt
SPECS="configG:ab_prev config2:ab_prev config4:ab_prev config5:ab_prev" REPS="1 2" timeout -k 10 900 bash tools/exp/ab_session.sh > gpurun_out/s24_ab.txt 2>&1; cat gpurun_out/s24_ab.txt
