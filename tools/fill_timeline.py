"""c5fir step timeline from a rocprofv3 kernel trace: per step (from its first converter launch to its
last render's end) the render launches, the gaps between them and the fill before the first"""
import csv, glob, sys
d = sys.argv[1]
f = glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0].replace('void ', ''))
              for r in csv.DictReader(open(f)))
k3 = [r for r in rows if 'render_rowc' in r[2]]
# a step starts at the first converter launch after an icw_advance
adv = [r[0] for r in rows if r[2].startswith('icw_advance')]
out = []
for a0, a1 in zip(adv, adv[1:]):
    ks = [r for r in k3 if a0 < r[0] < a1]
    if len(ks) < 3:
        continue
    first = min(r[0] for r in rows if a0 < r[0] < a1 and 'fir_graph' in r[2])
    busy = sum(e - s for s, e, _ in ks)
    gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
    span = ks[-1][1] - first
    out.append(f"step: span {span/1e6:.3f} ms, render busy {busy/1e6:.3f} ms, fill {(ks[0][0]-first)/1e3:.0f} us, "
               f"gaps {sum(gaps)/1e3:.0f} us\n  render launches (us): {[round((e-s)/1e3) for s, e, _ in ks]}\n"
               f"  gaps before each next one (us): {[round(g/1e3) for g in gaps]}")
print('\n'.join(out[-2:]))
last = out and [r for r in rows if adv[-2] < r[0] < adv[-1]]
if last:
    t0 = last[0][0]
    print('  last step, every kernel (start us, duration us, name):')
    for s, e, n in last:
        print(f'    {(s-t0)/1e3:8.0f} {(e-s)/1e3:6.0f}  {n}')
