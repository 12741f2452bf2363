# Diagnostic session: bs16 parity, mode timings, then the ablation builds.
set -e
mkdir -p gpurun_out
B=boringssl_amd/csrc/build
[ -n "${NOTEST:-}" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "bs16" -x -q --timeout 120 --timeout-method thread > gpurun_out/bs16test.log 2>&1
[ -n "${NOTEST:-}" ] || timeout -k 10 120 python tools/exp/modes.py table bs16 bs table > gpurun_out/v_main.log 2>&1
for v in ${VARS:-ablate1 ablate2 ablate3 ablate4}; do
  BSSL_AMD_LIB=$PWD/$B/$v/libbssl_amd.so timeout -k 10 120 python tools/exp/modes.py table > gpurun_out/v_$v.log 2>&1
done
