set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1200 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
for al in 128 16; do
  BSSL_AMD_ALIGN=$al timeout -k 10 300 python bench.py --config config3 --no-cpu-baseline > gpurun_out/b_config3_a$al.log 2>&1 || exit 1
  echo "config3 align=$al $(grep -o '"value": [0-9.]*\|"parity": "[^"]*"' gpurun_out/b_config3_a$al.log | tr '\n' ' ')"
done
for a in chacha20-poly1305 xchacha20-poly1305; do timeout -k 10 300 python tools/iov_bench.py --aead $a --records 1048576 --len 1350 2>&1 | grep "^{"; done
