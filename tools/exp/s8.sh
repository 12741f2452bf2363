set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pers4; do
BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/ab_$v/libbssl_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "chacha or uniform or baseline_config_digest" --timeout 300 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || { tail -20 gpurun_out/t_$v.log; exit 1; }
tail -1 gpurun_out/t_$v.log
done
SPECS="config3:ab_pers4,ab_pers8 config3x:ab_pers4,ab_pers8" REPS="1 2" timeout -k 10 900 bash tools/exp/ab_session.sh > gpurun_out/ab_pers.txt 2>&1; cat gpurun_out/ab_pers.txt
