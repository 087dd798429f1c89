set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lt && cd gpurun_out/lt
python3 -c "
import sys; sys.path.insert(0,'../../tests'); sys.path.insert(0,'../../tla-raft_amd'); sys.path.insert(0,'../../oracle'); sys.path.insert(0,'../..')
from test_host import cfg_text
open('RaftSeeded.cfg','w').write(cfg_text(E=2,R=3,vals='v1'))
"
export RMC_SKIP_SPEC_CHECK=1
timeout -k 10 120 ../../tla-raft_amd/build/raftmc -deadlock -config RaftSeeded.cfg RaftSeeded.tla > one.txt 2> one.err; echo "one rc $?"
timeout -k 10 120 ../../tla-raft_amd/build/raftmc -gpus 1 -onerank -shardmin 1 -deadlock -config RaftSeeded.cfg RaftSeeded.tla > rk.txt 2> rk.err; echo "rk rc $?"
diff one.txt rk.txt | head -40
