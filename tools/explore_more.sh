set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for c in "3 1 3 3" "5 1 2 3" "4 1 2 3" "3 2 2 1"; do
  set -- $c
  echo "== $c"
  timeout -k 10 200 python -u tools/explore.py $1 $2 $3 $4 --budget 150 > gpurun_out/explore_n$1_v$2_e$3_r$4.log 2>&1
  rc=$?; tail -3 gpurun_out/explore_n$1_v$2_e$3_r$4.log
  if [ $rc -ne 0 ] && ! grep -q "out of memory" gpurun_out/explore_n$1_v$2_e$3_r$4.log; then echo "rc=$rc"; exit 1; fi
done
