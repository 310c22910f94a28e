"""Per-kernel averages of rocprofv3 --pmc counters (counter_collection.csv),
kernels named as tools/trace_ops.py names them.
    python tools/pmc_summary.py run_counter_collection.csv [name-filter]"""
import csv
import sys
from collections import defaultdict

from trace_ops import name_of


def main():
  flt = sys.argv[2] if len(sys.argv) > 2 else ''
  acc = defaultdict(lambda: defaultdict(float))
  disp = defaultdict(set)
  for r in csv.DictReader(open(sys.argv[1])):
    n = name_of(r['Kernel_Name'])
    if flt not in n:
      continue
    acc[n][r['Counter_Name']] += float(r['Counter_Value'])
    disp[n].add(r['Dispatch_Id'])
  for n, c in acc.items():
    k = len(disp[n])
    print('%s  (%d dispatches)' % (n[:110], k))
    print('   ' + '  '.join('%s=%.4g' % (cn, v / k) for cn, v in sorted(c.items())))


if __name__ == '__main__':
  main()
