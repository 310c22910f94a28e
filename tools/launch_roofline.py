"""Per-launch roofline of the Rainbow step (bench.py's default schedule, B = 32, 9 actions x
51 atoms): each of the step's 11 launches with its duration (rocprofv3 --kernel-trace), its
HBM-side bytes (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, one counter per pass), its
algorithmic FLOPs, its fraction of the binding resource, and its counted bytes against its
algorithmic bytes (every tensor it reads once, every tensor it writes once: ALGO).

    rocprofv3 --kernel-trace -d T -o run -- python3 bench.py --skip-cpu-baseline --skip-configs
    rocprofv3 --pmc FETCH_SIZE -d F -o run --output-format csv -- python3 bench.py <same, short>
    rocprofv3 --pmc WRITE_SIZE -d W -o run --output-format csv -- python3 bench.py <same, short>
    python tools/launch_roofline.py T/run_results.db F W > table.md

Steps are cut at the loss kernel (k_c51), which starts every step; launch i of a step is
the i-th dispatch after it.  Per launch: the median duration over the traced steps, the mean
counters over the PMC steps (dispatches are serialised under --pmc, so the counts are per
launch).  FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: gfx950 reports half the bytes of
16-B-per-lane reads, which the GEMM operand fetches and the Adam riders are); WRITE_SIZE is
taken as is (exact for 16-B stores; the GEMM epilogues' 4-B stores are uncalibrated).  Both
count Infinity-Cache hits (guide): "bytes" are L2-miss traffic, HBM or MALL.
"""
import csv
import glob
import os
import re
import sqlite3
import statistics
import sys

HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md
FP32_MFMA_PEAK = 157.3e12  # FLOP/s, v_mfma_f32_32x32x2_f32 dense

B, A, N = 32, 9, 51
NO = A * N
# MACs of each product (per batch of B)
C1 = 21 * 21 * 32 * (8 * 8 * 4) * B
C2 = 11 * 11 * 64 * (4 * 4 * 32) * B
C3 = 11 * 11 * 64 * (3 * 3 * 64) * B
FC1 = 7744 * 512 * B
FC2 = 512 * NO * B
# dW = x^T dy (+ the bias ones-column), dX = dy W
DW = {'fc2': NO * 513 * B, 'fc1': 512 * 7745 * B, 'conv3': 64 * 577 * 121 * B,
      'conv2': 64 * 513 * 121 * B, 'conv1': 32 * 257 * 441 * B}
DX = {'fc1': 7744 * 512 * B, 'conv3': 121 * 64 * 576 * B,
      'conv2': 21 * 21 * 32 * (2 * 2 * 64) * B}   # sub-pixel classes: 2 x 2 taps x 64
DH = 51 * 512 * B                                      # d h = dlogits . W2 (chosen action)

# Algorithmic bytes: every tensor a launch reads once, every tensor it writes once (fp32; TF1
# Adam in an epilogue reads and writes p, m, v: 3 + 3 times the weights).
STATE = B * 84 * 84 * 4 * 4                 # a gathered state stack, NHWC fp32
A1, A2, A3 = B * 441 * 32 * 4, B * 121 * 64 * 4, B * 121 * 64 * 4
H, DOUT = B * 512 * 4, B * NO * 4
W_C1, W_C2, W_C3 = (8 * 8 * 4 * 32 + 32) * 4, (4 * 4 * 32 * 64 + 64) * 4, (3 * 3 * 64 * 64 + 64) * 4
W_FC1, W_FC2 = (7744 * 512 + 512) * 4, (512 * NO + NO) * 4
NZ3, NZ1 = 8, 28                            # split-K slabs (kSplitConvW, kSplitConv1W)
SLAB3, SLAB2, SLAB1 = NZ3 * 64 * 577 * 4, NZ3 * 64 * 513 * 4, NZ1 * 32 * 257 * 4
FC1_PARTS = 2 * 16 * B * 512 * 4            # fc1 split-K partials, both nets (kSplitFc1 16)
FC2_PARTS = 2 * 16 * B * NO * 4             # fc2 k-band partials, both nets (FcHeadOp::kBands)
FRAMES = 2 * B * 4 * 84 * 84                # the PER gather rider's frames in (two stacks out)
TREE = B * 21 * 8 * 2                       # a PER write-back or sample rider's tree path
ALGO = [  # (bytes read, bytes written) per launch, in LAUNCHES order
    (FC2_PARTS + W_FC2, H + DOUT),                                       # C: d h, dlogits
    (H + W_FC1 + A3, A3),                                                # B1: d a3
    (H + A3 + 3 * W_FC1 + A3 + W_C3 + A2 + DOUT + 3 * W_FC2 + TREE,     # B2 (d h, a3 once)
     3 * W_FC1 + A2 + 3 * W_FC2 + TREE),
    (A3 + A2 + A2 + W_C2 + A1 + TREE, SLAB3 + A1 + SLAB2),               # B3 (d a2, a1 once)
    (SLAB3 + A1 + STATE + FRAMES, W_C3 + SLAB1 + 2 * STATE),            # B4 + gather
    (SLAB2 + 3 * W_C2 + SLAB1 + 3 * W_C1 + 4 * W_C3 + STATE + W_C1,     # B5 + target conv1
     3 * W_C2 + 3 * W_C1 + 3 * W_C3 + A1),
    (STATE + W_C1, A1),                                                  # F1
    (2 * A1 + 2 * W_C2, 2 * A2),                                         # F2
    (2 * A2 + 2 * W_C3, 2 * A3),                                         # F3
    (2 * A3 + 2 * W_FC1, FC1_PARTS),                                     # F4
    (FC1_PARTS + 2 * W_FC2, 2 * H + FC2_PARTS),                          # F5
]
# counter scale factors (tools/micro/pmc_calib.hip, profiles/r5_roofline/pmc_calib.md)
FETCH_SCALE, WRITE_SCALE = 2.0, 1.0

# the step's launches in order from the loss kernel and what they compute
LAUNCHES = [
    ('C  k_c51', 'loss + d h', DH),
    ('B1', 'dX fc1', DX['fc1']),
    ('B2', 'dW fc1 / dW fc2, their Adam (epilogues) / dX conv3 + PER write-back',
     DW['fc1'] + DW['fc2'] + DX['conv3']),
    ('B3', 'dW conv3 / dX conv2 / dW conv2 + PER sample', DW['conv3'] + DX['conv2'] + DW['conv2']),
    ('B4', 'sum conv3 / dW conv1 + gather', DW['conv1']),
    ('B5', 'sum conv2/conv1 + Adam conv1-3 + target conv1', C1),
    ('F1', 'conv1', C1),
    ('F2', 'conv2 + target conv2', 2 * C2),
    ('F3', 'conv3 + target conv3', 2 * C3),
    ('F4', 'fc1 split-K, online + target', 2 * FC1),
    ('F5', 'fc1 sum + fc2 k-band partials, both nets', 2 * FC2),
]


def _steps(names, anchor='k_c51'):
  cuts = [i for i, n in enumerate(names) if anchor in n]
  return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b - a == len(LAUNCHES)]


def durations(db_path, skip=30):
  db = sqlite3.connect(db_path)
  rows = sorted(db.execute('select start, end, name from kernels'))
  names = [r[2] for r in rows]
  per = [[] for _ in LAUNCHES]
  for a, b in _steps(names)[skip:]:
    for i in range(len(LAUNCHES)):
      per[i].append((rows[a + i][1] - rows[a + i][0]) / 1e3)
  return [statistics.median(p) if p else float('nan') for p in per]


def counters(d, counter, skip=10):
  rows = []
  for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
      if r['Counter_Name'] == counter:
        rows.append((int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value'])))
  rows.sort()
  names = [r[1] for r in rows]
  per = [[] for _ in LAUNCHES]
  kn = [None] * len(LAUNCHES)
  for a, b in _steps(names)[skip:]:
    for i in range(len(LAUNCHES)):
      per[i].append(rows[a + i][2] * 1024.0)      # KiB -> bytes
      kn[i] = rows[a + i][1]
  return [statistics.mean(p) if p else float('nan') for p in per], kn


def short(n):
  n = re.sub(r'dq::cnn::|dq::|void ', '', n or '')
  return n[:60]


def main():
  dur = durations(sys.argv[1])
  fetch, kn = counters(sys.argv[2], 'FETCH_SIZE')
  write, _ = counters(sys.argv[3], 'WRITE_SIZE')
  print('| launch | work | us | GFLOP | TFLOP/s | frac fp32 MFMA | fetch MB (x%g) | write MB | '
        'TB/s | frac HBM | binding | algo MB (r + w) | measured / algo |' % FETCH_SCALE)
  print('|---|---|---|---|---|---|---|---|---|---|---|---|---|')
  tot = [0.0, 0.0, 0.0, 0.0]
  for (name, what, macs), t, f, w, k, (ar, aw) in zip(LAUNCHES, dur, fetch, write, kn, ALGO):
    fl = 2.0 * macs
    tf = fl / (t * 1e-6)
    f, w = FETCH_SCALE * f, WRITE_SCALE * w
    by = f + w
    bw = by / (t * 1e-6)
    fm, fh = tf / FP32_MFMA_PEAK, bw / HBM_PEAK
    tot[0] += t
    tot[1] += fl
    tot[2] += by
    tot[3] += ar + aw
    print('| %s | %s | %.1f | %.3f | %.1f | %.3f | %.2f | %.2f | %.2f | %.3f | %s | %.2f + %.2f | '
          '%.2f (r %.2f, w %.2f) |' % (
              name, what, t, fl / 1e9, tf / 1e12, fm, f / 1e6, w / 1e6, bw / 1e12, fh,
              'MFMA' if fm > fh else 'HBM', ar / 1e6, aw / 1e6, by / (ar + aw), f / ar, w / aw))
  print('| step | | %.1f | %.3f | %.1f | %.3f | | | %.2f | %.3f | | %.2f | %.2f |' % (
      tot[0], tot[1] / 1e9, tot[1] / (tot[0] * 1e-6) / 1e12, tot[1] / (tot[0] * 1e-6) / FP32_MFMA_PEAK,
      tot[2] / (tot[0] * 1e-6) / 1e12, tot[2] / (tot[0] * 1e-6) / HBM_PEAK, tot[3] / 1e6,
      tot[2] / tot[3]))
  print()
  for (name, _, _), k in zip(LAUNCHES, kn):
    print('- %s: `%s`' % (name, short(k)))


if __name__ == '__main__':
  main()
