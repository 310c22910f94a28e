"""Reads the two rocprofv3 --pmc passes over tools/micro/pmc_calib.hip and prints, per kernel,
FETCH_SIZE and WRITE_SIZE (in bytes; the counters report KiB) against the bytes the kernel
moves: the calibration factors tools/launch_roofline.py applies.

    python tools/pmc_calib.py <FETCH_SIZE dir> <WRITE_SIZE dir>
"""
import collections
import csv
import glob
import os
import statistics
import sys

MIB = 1 << 20
# kernel -> (algorithmic bytes read, written)
EXPECT = {
    'k_read4': (512 * MIB, 0),
    'k_read16': (512 * MIB, 0),
    'k_read4_stride2': (256 * MIB, 0),      # bytes used; every line is touched
    'k_write4': (0, 512 * MIB),
    'k_write16': (0, 512 * MIB),
    'k_write4_half': (0, 256 * MIB),        # bytes stored; every line half written
    'k_bcast16': (1 * MIB, 0),              # one buffer read by 2048 workgroups
}


def read(d, counter):
  per = collections.defaultdict(list)
  for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
      if r['Counter_Name'] == counter:
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').strip()
        per[k].append(float(r['Counter_Value']) * 1024.0)
  return {k: statistics.median(v) for k, v in per.items()}


def main():
  fetch, write = read(sys.argv[1], 'FETCH_SIZE'), read(sys.argv[2], 'WRITE_SIZE')
  print('| kernel | bytes read | FETCH_SIZE | fetch / read | bytes written | WRITE_SIZE | write / written |')
  print('|---|---|---|---|---|---|---|')
  for k, (r, w) in EXPECT.items():
    f, wr = fetch.get(k, float('nan')), write.get(k, float('nan'))
    print('| %s | %.1f MB | %.1f MB | %s | %.1f MB | %.1f MB | %s |' % (
        k, r / 1e6, f / 1e6, '%.3f' % (f / r) if r else '-', w / 1e6, wr / 1e6,
        '%.3f' % (wr / w) if w else '-'))


if __name__ == '__main__':
  main()
