set -euo pipefail
mkdir -p gpurun_out
VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_single/libvo_hip.so timeout -k 10 300 python -m pytest tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py -x -q > gpurun_out/k3v_pytest.log 2>&1
bash tools/gpu_ba_variants.sh base single base single
