"""bench.py with schedule experiments applied (A/B runs; never the bench line): the same
protocol and JSON line, with the agent-class attributes / constructor overrides below set
first.  The line's "build.overrides" names what was changed.

    python tools/bench_ab.py [--fuse-opt 0|1] [--ride 0|1] [--split-c51 0|1] [--branch-first]
                             [--chunk-steps K] [--rider-launches a,b,c] [--sample-launch L]
                             [--comm-priority P] -- <bench.py arguments>
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  argv = sys.argv[1:]
  rest = []
  if '--' in argv:
    i = argv.index('--')
    argv, rest = argv[:i], argv[i + 1:]
  ap = argparse.ArgumentParser()
  ap.add_argument('--fuse-opt', type=int, default=None,
                  help='DQNAgent fuse_optimizer (0/1)')
  ap.add_argument('--ride', type=int, default=None, help='DQNAgent ride_replay (0/1)')
  ap.add_argument('--split-c51', type=int, default=None,
                  help='RainbowAgent.split_c51 (0/1): the C51 target half riding in the forward')
  ap.add_argument('--branch-first', action='store_true',
                  help='N > 1: capture the fc bucket\'s branch before the backward tail')
  ap.add_argument('--chunk-steps', type=int, default=None,
                  help='DQNAgent._UNROLL: gradient steps per learner-loop HIP graph')
  ap.add_argument('--rider-launches', default=None,
                  help='DQNAgent.rider_launches, e.g. 2,3,4 (PER write-back, sample, gather)')
  ap.add_argument('--sample-launch', type=int, default=None,
                  help='DQNAgent.sample_launch (2/3)')
  ap.add_argument('--comm-priority', type=int, default=None,
                  help='DQNAgent.comm_priority (0 / -1): the N > 1 comm stream\'s HIP priority')
  a = ap.parse_args(argv)
  import bench
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  ov = {}
  if a.fuse_opt is not None:
    ov['fuse_optimizer'] = bool(a.fuse_opt)
  if a.ride is not None:
    ov['ride_replay'] = bool(a.ride)
  if a.split_c51 is not None:
    RainbowAgent.split_c51 = bool(a.split_c51)
    ov['RainbowAgent.split_c51'] = bool(a.split_c51)
  if a.branch_first:
    DQNAgent.branch_first = True
    ov['DQNAgent.branch_first'] = True
  if a.chunk_steps is not None:
    DQNAgent._UNROLL = int(a.chunk_steps)
    ov['DQNAgent._UNROLL'] = int(a.chunk_steps)
  if a.rider_launches is not None:
    DQNAgent.rider_launches = tuple(int(x) for x in a.rider_launches.split(','))
    ov['DQNAgent.rider_launches'] = DQNAgent.rider_launches
  if a.sample_launch is not None:
    DQNAgent.sample_launch = int(a.sample_launch)
    ov['DQNAgent.sample_launch'] = int(a.sample_launch)
  if a.comm_priority is not None:
    DQNAgent.comm_priority = int(a.comm_priority)
    ov['DQNAgent.comm_priority'] = int(a.comm_priority)
  # class attributes are not constructor arguments: only the real kwargs go to build_agent
  bench.CLASS_OVERRIDES = {k: v for k, v in ov.items() if '.' in k}
  bench.AGENT_OVERRIDES = {k: v for k, v in ov.items() if '.' not in k}
  bench.main(rest)


if __name__ == '__main__':
  main()
