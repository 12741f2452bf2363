# Open-path A/B (tag compare): GCM config 2 and ChaCha config 3, --op open.
set -e
mkdir -p gpurun_out
B=boringssl_amd/csrc/build
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config config2 --op open --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/o_c2_main_$rep.log 2>&1
  BSSL_AMD_LIB=$PWD/$B/ab_oldgcm/libbssl_amd.so timeout -k 10 200 python bench.py --config config2 --op open --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/o_c2_old_$rep.log 2>&1
  timeout -k 10 200 python bench.py --config config3 --op open --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/o_c3_main_$rep.log 2>&1
  BSSL_AMD_LIB=$PWD/$B/ab_oldcha/libbssl_amd.so timeout -k 10 200 python bench.py --config config3 --op open --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/o_c3_old_$rep.log 2>&1
done
