# A/B of an environment switch ($1 = variable): bitwise teacher-forced logits (tools/debug/ab_logits.py) and
# rocprofv3 kernel stats of the 128-clip bench line at $1=0 and $1=1
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
V=$1
env $V=0 timeout -k 10 200 python tools/debug/ab_logits.py old && env $V=1 timeout -k 10 200 python tools/debug/ab_logits.py new || exit 1
python3 -c "
import numpy as np; a=np.load('gpurun_out/ab_old.npy'); b=np.load('gpurun_out/ab_new.npy')
print('logits bitwise equal:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'max |diff|', float(np.abs(a-b).max()))"
export $V=0; bash tools/debug/prof_lines.sh e0_b128 "--steps 2 --warmup 1" || exit 1
export $V=1; bash tools/debug/prof_lines.sh e1_b128 "--steps 2 --warmup 1" || exit 1
