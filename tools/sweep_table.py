"""Tabulate a tools/_sweep_wgrad.sh log: best (tile, split) per layer and the full grid."""
import collections
import re
import sys

cur = None
res = collections.defaultdict(dict)
for line in open(sys.argv[1]):
    m = re.match(r'== (\d+),(\d+) ks (\d+)', line)
    if m:
        cur = (int(m.group(1)), int(m.group(2)), int(m.group(3)))
        continue
    m = re.match(r'(\w+)\s+[\d.]+ GF \| wgrad ([\d.]+) ms (\d+) TF/s', line)
    if m and cur:
        res[m.group(1)][cur] = (float(m.group(2)), int(m.group(3)))
for layer, d in res.items():
    best = sorted(d.items(), key=lambda kv: kv[1][0])[:3]
    print(layer, [(k, v[0], v[1]) for k, v in best])
    cfgs = sorted({(k[0], k[1]) for k in d}, reverse=True)
    for cfg in cfgs:
        print("     ", cfg, " ".join("%d:%.3f" % (k[2], v[0]) for k, v in sorted(d.items()) if (k[0], k[1]) == cfg))
