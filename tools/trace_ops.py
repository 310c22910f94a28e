"""Average duration per kernel (grouped launches named by their ops) from a
rocprofv3 --kernel-trace CSV.   python tools/trace_ops.py run_kernel_trace.csv [N]"""
import csv
import re
import sys
from collections import defaultdict


def name_of(n):
  n = re.sub(r'dq::cnn::|dq::|void ', '', n)
  if n.startswith('k_grouped'):
    ops = []
    for m in re.finditer(r'(GemmOp<(\d+), (\d+), (\d+), (\w+)(?:<[^>]*(?:<[^>]*>)?[^>]*>)?, (\w+)'
                         r'(?:<[^>]*(?:<[^>]*>)?[^>]*>)?, (\w+)|ReduceOp<(\w+)|SubPix|AdamOp|RiderOp'
                         r'|FcHeadOp)', n):
      if m.group(1).startswith('GemmOp'):
        ops.append('G%s%s%s:%s/%s/%s' % (m.group(2), m.group(3), m.group(4), m.group(5),
                                          m.group(6), m.group(7)))
      elif m.group(8):
        ops.append('Sum:' + m.group(8))
      else:
        ops.append(m.group(1).replace('Op', ''))
    # the kernel name repeats the op list in its parameter types: keep the first half
    ops = ops[:max(1, len(ops) // 2)]
    return 'group[' + ' | '.join(ops) + ']'
  n = re.sub(r'Conv<(\d+), \d+, \d+, (\d+), [^>]*>', r'C\1k\2', n)
  return n.split('(')[0][:90]


def main():
  rows = list(csv.DictReader(open(sys.argv[1])))
  top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
  agg = defaultdict(list)
  for r in rows:
    agg[name_of(r['Kernel_Name'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
  print('%6s %8s %9s  %s' % ('count', 'avg_us', 'total_us', 'kernel'))
  for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print('%6d %8.2f %9.1f  %s' % (len(v), sum(v) / len(v), sum(v), k))


if __name__ == '__main__':
  main()
