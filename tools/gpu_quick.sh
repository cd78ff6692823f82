set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ba.py tests/test_gpu_dropin.py -x -q > gpurun_out/k3_pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/k3_bench.json 2> gpurun_out/k3_bench.err
VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > gpurun_out/k3_stamps.txt 2>&1
echo ok
