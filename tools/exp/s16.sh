set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/prof CONFIGS="config3 config3x" PASSES="stats pmc" bash tools/profile.sh > gpurun_out/prof_steps.txt 2>&1 || { tail gpurun_out/prof_steps.txt; exit 1; }
tail -2 gpurun_out/prof_steps.txt
bash tools/exp/s15.sh
