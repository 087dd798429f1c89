#!/bin/bash
# stress a library / env variant of the W=2 shard-min-40 multirank cases; stop at a time limit
O=gpurun_out/$1; shift; N=$1; shift
mkdir -p $O
fails=0
for i in $(seq 1 $N); do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread -k "identical and 40" > $O/mr$i.log 2>&1
  rc=$?
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "TIMEOUT $i"; exit 1; fi
  if [ $rc -ne 0 ]; then fails=$((fails+1)); echo "FAIL $i"; grep -E "^E " $O/mr$i.log | head -3 | cut -c1-300; fi
done
echo "$O: $fails failures in $N runs"
