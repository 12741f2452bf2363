# Round 5: FETCH_SIZE / WRITE_SIZE calibration copies at the bench geometries
# (tools/micro/calib_copy, tools/profile.sh "calib" pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5final}/prof CONFIGS="" PASSES="calib" bash tools/profile.sh
