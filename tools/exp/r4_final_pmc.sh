# Round-4 final evidence (part 2): PMC passes (FETCH_SIZE, WRITE_SIZE, the
# SQ/GRBM busy set; one rocprofv3 run each) of the bench commands.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4final/prof CONFIGS="${CONFIGS:-config2 configG config3 config4 config5}" PASSES="pmc" bash tools/profile.sh
