set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_aead_api_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/api_tests.log 2>&1 || { tail -30 gpurun_out/api_tests.log; exit 1; }
tail -1 gpurun_out/api_tests.log
timeout -k 10 300 python tools/latency_bench.py > gpurun_out/lat_mapped.json 2>&1 && tail -1 gpurun_out/lat_mapped.json
BSSL_AMD_ONE_RECORD_MAP_MAX=0 timeout -k 10 300 python tools/latency_bench.py > gpurun_out/lat_copy.json 2>&1 && tail -1 gpurun_out/lat_copy.json
SPECS="config3:ab_sdwa,ab_unr5,ab_unr2,ab_ntl,ab_prio0,ab_l2" timeout -k 10 1000 bash tools/exp/ab_session.sh > gpurun_out/ab.txt 2>&1; cat gpurun_out/ab.txt
