set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPECS="config3:ab_w4 config3x:ab_w4" REPS="1 2" timeout -k 10 900 bash tools/exp/ab_session.sh > gpurun_out/ab_w4.txt 2>&1; cat gpurun_out/ab_w4.txt
