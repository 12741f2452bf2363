set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "chacha or uniform or iovec" --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for L in l2 l2w3; do BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/ab_$L/libbssl_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "chacha and not iovec" --timeout 300 --timeout-method thread > gpurun_out/t_$L.log 2>&1; tail -1 gpurun_out/t_$L.log; done
SPECS="config3:ab_l2,ab_l2w3 config3x:ab_l2,ab_l2w3" REPS="1 2 3" timeout -k 10 1000 bash tools/exp/ab_session.sh > gpurun_out/ab.txt 2>&1; cat gpurun_out/ab.txt
