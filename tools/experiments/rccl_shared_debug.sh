cd $GRAFT_REPO_ROOT
export QUEST_BACKEND=hip QUEST_COMM=rccl QUEST_RCCL_SHARED_GPU=1 QUEST_COMM_TIMEOUT=30 QUEST_TEST_STACKS=50 NCCL_DEBUG=WARN PYTHONPATH=$GRAFT_REPO_ROOT
python - <<'PY'
import os, sys
sys.path.insert(0, "tests")
from quest_amd.parallel import spawn_local
res = spawn_local(["tests/dist_worker.py", "calculations", "/tmp/calc.npz"], 2, env_extra={}, timeout=80)
for r, p in enumerate(res):
    print("rank", r, "rc", p.returncode)
    print(p.stdout[-3000:])
    print(p.stderr[-6000:])
PY
