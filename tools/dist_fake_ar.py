"""One-rank RCCL bench with the fc bucket's all-reduce replaced by an in-place multiply on
the comm stream (a torch kernel of similar bytes): tells the HIP graph's fork / join cost
apart from RCCL's own launch behaviour.  An experiment, not the bench line.
    python tools/dist_fake_ar.py [bench args]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dopamine_amd.agents.dqn import dqn_agent  # noqa: E402

dqn_agent.DQNAgent._ar_fc = lambda self, t: t.mul_(1.0)
sys.argv = [sys.argv[0], '--force-dist', '--zero', '0', '--skip-cpu-baseline', '--skip-configs'] + sys.argv[1:]
bench.main()
