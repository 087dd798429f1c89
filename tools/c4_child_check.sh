set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k configs3 --timeout 240 --timeout-method thread > gpurun_out/t_c4.log 2>&1 || { tail -20 gpurun_out/t_c4.log; exit 1; }
tail -2 gpurun_out/t_c4.log
RANK=0 WORLD_SIZE=1 MASTER_PORT=29611 timeout -k 10 300 python -u bench.py --sharded-child --sharded-out gpurun_out/c4_mem.json --child-workload c4 --child-budget 200 > gpurun_out/c4_mem.log 2>&1 || { tail -20 gpurun_out/c4_mem.log; exit 1; }
cat gpurun_out/c4_mem.json; echo
RANK=0 WORLD_SIZE=1 MASTER_PORT=29631 timeout -k 10 200 python -u bench.py --sharded-child --sharded-out gpurun_out/c4_budget.json --child-workload c4 --child-budget 35 > gpurun_out/c4_budget.log 2>&1 || { tail -20 gpurun_out/c4_budget.log; exit 1; }
cat gpurun_out/c4_budget.json; echo
