import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'adam' in r['Kernel_Name']]
s, e = idx[-2] + 1, idx[-1] + 1
if e < len(rows) and 'transpose' in rows[e]['Kernel_Name']:
    pass
t0 = int(rows[s]['Start_Timestamp'])
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = {}
for r in rows[s:e + 1]:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    import re
    nm = r['Kernel_Name'].replace('gm2::(anonymous namespace)::', '').replace('void ', '')
    k = re.sub(r'\(.*$', '', nm.split('(gm2')[0])[:60]
    if 'Cfg<' in nm:
        k += '<' + re.search(r'Cfg<([^>]*)>', nm).group(1) + '>'
    tot[k] = tot.get(k, 0) + d
    if d > thr:
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {d:8.1f}us grid={r.get('Grid_Size_X', '?')} {k}")
print('step span us', (int(rows[e]['End_Timestamp']) - t0) / 1e3)
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"{v:9.1f} us  {k}")
