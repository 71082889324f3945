#!/usr/bin/env python3
"""L2 (TCC) hits, misses and requests per stage kernel from a rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum
TCC_REQ_sum pass: python scripts/tcc_summary.py <run_counter_collection.csv>"""
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(__import__('sys').argv[1])):
    n = r['Kernel_Name'].split('(')[0].replace('void ', '')
    if 'merson' not in n: continue
    agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, d in agg.items():
    h = sum(d['TCC_HIT_sum'])/len(d['TCC_HIT_sum']); m = sum(d['TCC_MISS_sum'])/len(d['TCC_MISS_sum']); q = sum(d['TCC_REQ_sum'])/len(d['TCC_REQ_sum'])
    print(f"{n:35s} launches {len(d['TCC_HIT_sum']):3d} req {q/1e6:8.2f} M  hit {h/1e6:8.2f} M  miss {m/1e6:8.2f} M  hit rate {h/(h+m):.3f}")
