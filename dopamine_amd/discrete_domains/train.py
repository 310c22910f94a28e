"""Entry point (reference dopamine/discrete_domains/train.py):

    python -m dopamine_amd.discrete_domains.train --base_dir /tmp/cartpole \\
        --gin_files dopamine_amd/agents/dqn/configs/dqn_cartpole.gin \\
        [--gin_bindings 'Runner.num_iterations = 2']
"""
import argparse
import logging

from dopamine_amd.discrete_domains import run_experiment


def main(argv=None):
  ap = argparse.ArgumentParser()
  ap.add_argument('--base_dir', required=True,
                  help='Base directory to host all required sub-directories.')
  ap.add_argument('--gin_files', action='append', default=[],
                  help='Paths to gin configuration files.')
  ap.add_argument('--gin_bindings', action='append', default=[],
                  help='Gin bindings overriding the files (e.g. "DQNAgent.epsilon_train=0.1").')
  args = ap.parse_args(argv)
  logging.getLogger().setLevel(logging.INFO)
  run_experiment.load_gin_configs(args.gin_files, args.gin_bindings)
  runner = run_experiment.create_runner(args.base_dir)
  runner.run_experiment()
  return runner


if __name__ == '__main__':
  main()
