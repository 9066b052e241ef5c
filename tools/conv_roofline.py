import csv, json
conv = json.load(open('/tmp/convshapes.json'))
rows = list(csv.DictReader(open('/root/repo/gpurun_out/prof3/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i,r in enumerate(rows) if 'sgd_flat' in r['Kernel_Name']]
step = rows[idx[-2]+1: idx[-1]+1]
ig = [r for r in step if 'igemm' in r['Kernel_Name']]
j = 0; out = []
for (mode, gm, gn, gk, s, R) in conv:
    n = 1
    if mode == 'dgrad' and s == 2: n = 1 if R == 1 else 4
    d = sum((int(r['End_Timestamp'])-int(r['Start_Timestamp'])) for r in ig[j:j+n]) / 1e3
    tiles = ig[j]['Kernel_Name'].split('<')[1].split('>')[0]
    j += n
    fl = 2.0*gm*gn*gk
    if mode == 'dgrad' and s == 2: fl /= 4 if R == 1 else 1  # useful flops only (1x1 s2 dgrad rows)
    if mode == 'wgrad': by = 2*(gk*gm + gk*gn) + 4*gm*gn
    else: by = 2*(gm*gk/ (R*R) + gm*gn) if R>1 else 2*(gm*gk + gm*gn)
    out.append((d, mode, gm, gn, gk, s, R, fl/d/1e6, by/d/1e3, tiles))
print("matched", j, "of", len(ig))
tot = sum(o[0] for o in out)
print(f"total conv us {tot:.0f}")
agg = {}
for o in out:
    k = (o[1], o[2], o[3], o[4], o[5], o[6]); agg.setdefault(k, [0, 0, o[7], o[8], o[9]]); agg[k][0] += o[0]; agg[k][1] += 1
for k, v in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"{v[0]:8.0f}us x{v[1]:2d} {k[0]:6s} gm={k[1]:8d} gn={k[2]:5d} gk={k[3]:7d} s={k[4]} R={k[5]}  {v[2]:6.0f} TF/s  {v[3]:6.2f} TB/s  <{v[4]}>")
