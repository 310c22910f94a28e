"""One-rank RCCL bench with the conv bucket's all-reduce over torch.distributed's second
communicator (torch's own RCCL) and the fc bucket's over the learner's RcclComm: tells
whether the fc all-reduce's late start (profiles/r3_dist) comes from one RCCL instance
ordering its two communicators' kernels.  An experiment, not the bench line.
    python tools/dist_mixed.py [bench args]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dopamine_amd import parallel  # noqa: E402
from dopamine_amd.agents.dqn import dqn_agent  # noqa: E402

dqn_agent.DQNAgent._ar_conv = lambda self, t, second: parallel.allreduce_mean_(
    t, self._conv_group() if second else self._pg)
sys.argv = [sys.argv[0], '--force-dist', '--zero', '0', '--skip-cpu-baseline', '--skip-configs'] + sys.argv[1:]
bench.main()
