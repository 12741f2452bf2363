# Bench lines for every BASELINE config with the current build (GPU box).
set -e
mkdir -p gpurun_out
for c in config3 config3x config4 config5 configS; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline > gpurun_out/cfg_$c.log 2>&1
done
timeout -k 10 300 python bench.py --config config2 --op open --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/cfg_config2_open.log 2>&1
timeout -k 10 300 python bench.py --config config3 --op open --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/cfg_config3_open.log 2>&1
