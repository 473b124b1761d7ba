set -eo pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_l0.log 2>&1
bash tools/config_lines.sh l0
LBIC_L0CACHE=0 bash tools/config_lines.sh nol0
