# Diagnostic session: same-box A/B of library builds on config 2 (modes.py),
# optionally preceded by the GCM GPU parity tests of the main build.
set -e
mkdir -p gpurun_out
B=boringssl_amd/csrc/build
[ -n "${NOTEST:-}" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "${TESTK:-gcm}" -x -q --timeout 120 --timeout-method thread > gpurun_out/test.log 2>&1
for rep in 1 2; do
  timeout -k 10 120 python tools/exp/modes.py table > gpurun_out/v_main_$rep.log 2>&1
  for v in ${VARS:-}; do
    BSSL_AMD_LIB=$PWD/$B/$v/libbssl_amd.so timeout -k 10 120 python tools/exp/modes.py table > gpurun_out/v_${v}_$rep.log 2>&1
  done
done
