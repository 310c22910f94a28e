"""Workload for the gather kernel's PMC traffic passes (MI355X_MICROARCH.md, HBM).

Runs k_gather_nhwc4 on a full synthetic 1M-transition buffer with FRESH random
valid indices per launch (cold frames, as in the learner step), at B = 32 (the
bench workload) and at B = 1024 (calibration: distinct frames, so the unique
read bytes are known).  Run once per counter:

  rocprofv3 --pmc FETCH_SIZE -d OUT/fetch -o run --output-format csv -- python3 tools/gather_traffic.py
  rocprofv3 --pmc WRITE_SIZE -d OUT/write -o run --output-format csv -- python3 tools/gather_traffic.py
  python3 tools/gather_traffic.py --summarize OUT  > profiles/r1_gather_traffic.json
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LAUNCHES = 64
OBS = 84 * 84
STACK = 4


def run():
  import torch
  import bench
  from dopamine_amd import _lib
  from dopamine_amd.replay_memory.prioritized_replay_buffer import OutOfGraphPrioritizedReplayBuffer
  dev = torch.device('cuda', 0)
  C = 1_000_000
  mem = OutOfGraphPrioritizedReplayBuffer((84, 84), STACK, C, 32, update_horizon=3, device=dev)
  bench.fill_synthetic(mem, 9, seed=1)
  torch.cuda.synchronize()
  g = torch.Generator(device='cpu').manual_seed(3)
  for B in (32, 1024):
    out = mem._alloc_batch(B, _lib.LAYOUT_F32_NHWC)
    idx = torch.randint(STACK, C - 4, (LAUNCHES, B), generator=g, dtype=torch.int32).to(dev)
    for i in range(LAUNCHES):
      mem._gather(idx[i], B, _lib.LAYOUT_F32_NHWC, out)
    torch.cuda.synchronize()
    del out


def _per_launch(d, counter):
  """{batch: mean counter value per k_gather_nhwc4 dispatch}, dispatches in order:
  the first LAUNCHES are B = 32, the next LAUNCHES are B = 1024."""
  vals = []
  for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
      if 'k_gather_nhwc4' in r['Kernel_Name'] and r['Counter_Name'] == counter:
        vals.append((int(r['Dispatch_Id']), float(r['Counter_Value'])))
  vals.sort()
  per = {}
  for did, v in vals:
    per[did] = per.get(did, 0.0) + v          # sum over XCD/instance rows of one dispatch
  seq = [per[k] for k in sorted(per)]
  assert len(seq) == 2 * LAUNCHES, 'expected %d gather dispatches, got %d' % (2 * LAUNCHES, len(seq))
  return {32: sum(seq[:LAUNCHES]) / LAUNCHES, 1024: sum(seq[LAUNCHES:]) / LAUNCHES}


def summarize(d):
  fetch = _per_launch(os.path.join(d, 'fetch'), 'FETCH_SIZE')
  write = _per_launch(os.path.join(d, 'write'), 'WRITE_SIZE')
  kib = 1024.0   # rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB
  algo_read = {B: B * 2 * STACK * OBS for B in (32, 1024)}
  algo_write = {B: B * 2 * STACK * OBS * 4 for B in (32, 1024)}
  # calibration (guide: dword-per-lane reads are uncalibrated): at B = 1024 the
  # frames are distinct random 7 KB blocks of a 7 GB store, so the unique read
  # bytes are the algorithmic ones
  cal = algo_read[1024] / (fetch[1024] * kib)
  out = {
      'kernel': 'k_gather_nhwc4', 'launches_per_batch': LAUNCHES,
      'fetch_size_kib_per_launch': fetch, 'write_size_kib_per_launch': write,
      'fetch_calibration_factor': cal,
      'hbm_read_bytes_per_launch': {B: fetch[B] * kib * cal for B in fetch},
      'hbm_write_bytes_per_launch': {B: write[B] * kib for B in write},
      'algo_read_bytes': algo_read, 'algo_write_bytes': algo_write,
  }
  out['traffic_bytes_per_launch'] = {
      B: out['hbm_read_bytes_per_launch'][B] + out['hbm_write_bytes_per_launch'][B] for B in fetch}
  print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == '__main__':
  ap = argparse.ArgumentParser()
  ap.add_argument('--summarize', default=None)
  a = ap.parse_args()
  if a.summarize:
    summarize(a.summarize)
  else:
    run()
