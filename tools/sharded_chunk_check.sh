set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "rccl or sharded or golden_levels" > gpurun_out/t_big.log 2>&1 || { tail -20 gpurun_out/t_big.log; exit 1; }
tail -1 gpurun_out/t_big.log
RANK=0 WORLD_SIZE=1 MASTER_PORT=29650 timeout -k 10 700 python -u tools/sharded_legs_check.py gpurun_out/legs2.json > gpurun_out/legs2.log 2>&1 || { tail -5 gpurun_out/legs2.log; exit 1; }
tail -1 gpurun_out/legs2.log
