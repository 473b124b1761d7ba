set -eo pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python3 -u tools/decN_exp.py pool 384 4 > $O/decN_pool.log 2>&1
timeout -k 10 120 python3 -u tools/decN_exp.py raw 384 4 > $O/decN_raw.log 2>&1
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 -u tools/decN_exp.py raw 384 4 > $O/decN_raw_q8.log 2>&1
GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 -u tools/decN_exp.py raw 384 4 > $O/decN_raw_q16.log 2>&1
GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python3 -u tools/decN_exp.py raw 384 4 > $O/decN_raw_q2.log 2>&1
echo ok
