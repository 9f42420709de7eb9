"""Summarise the main loop of a kernel in a hipcc -S listing (diagnostic):
global loads GL, LDS writes DW / reads DR, smfmac/mfma M, vmcnt/lgkmcnt waits,
barriers.  usage: loopscan.py listing.s mangled_name [max_items]"""
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 200
i = s.index(name + ':')
body = s[i:s.index('.Lfunc_end', i)].split('\n')
st = [n for n, l in enumerate(body) if 'Loop Header' in l][0]
lab = body[st].split(':')[0].strip()
en = max(n for n, l in enumerate(body) if n > st and lab in l and 's_cbranch' in l)
out = []
for l in body[st:en + 1]:
    l = l.strip()
    if 's_waitcnt' in l or 's_barrier' in l or 'scratch' in l:
        out.append(l.split(';')[0].replace('s_waitcnt ', '').strip())
    elif l.startswith('global_load'): out.append('GL')
    elif l.startswith('ds_write'): out.append('DW')
    elif l.startswith('ds_read'): out.append('DR')
    elif 'mfma' in l: out.append('M')
comp, prev, cnt = [], None, 0
for o in out + [None]:
    if o == prev:
        cnt += 1
        continue
    if prev is not None:
        comp.append(prev + (f'x{cnt}' if cnt > 1 else ''))
    prev, cnt = o, 1
print(f'{en - st} lines:', ' '.join(comp[:lim]))
