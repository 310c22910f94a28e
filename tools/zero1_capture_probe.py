"""One-rank RCCL, ZeRO-1 with the slice's update on a second stream (comm -> comm_opt ->
comm), captured in the learner loop's chunk graphs -- over torch.distributed's collectives
(argv[1] == 'torch') or the learner's own communicators ('native').  Prints the outcome;
run each variant in its own process (round 2 saw a segfault in capture_end):
    python tools/zero1_capture_probe.py torch|native"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dopamine_amd import parallel  # noqa: E402
from tests.test_gpu_multirank import _agent, _run  # noqa: E402
from tests.test_gpu_rccl import _free_port  # noqa: E402

native = sys.argv[1] == 'native'
torch.cuda.set_device(0)
dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % _free_port(), rank=0,
                        world_size=1, device_id=torch.device('cuda', 0))
parallel.FORCE_COLLECTIVES = True
agent = _agent(dist.group.WORLD, 0, shard_optimizer=True, native_comm=native)
agent.zero_update_stream = True
print('capturing', sys.argv[1], flush=True)
flat = _run(agent, True).numpy()
print('captured chunks:', [k for k in agent._graph_sets if isinstance(k, tuple)], flush=True)
single = _run(_agent(None, 0), True).numpy()
print('bitwise equal to a single learner:', bool(np.array_equal(flat, single)), flush=True)
dist.destroy_process_group()
