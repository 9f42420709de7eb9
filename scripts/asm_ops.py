"""Memory ops / waits / branches of one kernel in a hipcc --cuda-device-only -S
listing (diagnostic).  usage: asm_ops.py listing.s name_substring [max_lines]"""
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
names = [l.split(':')[0] for l in s.split('\n') if ': ; @' in l and sub in l]
n = names[0]
i = s.index(n + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].split('\n')
out = []
for l in body:
    l = l.strip()
    if l.startswith(('s_waitcnt', 'global_load', 'ds_', 'global_store', 'buffer_', 's_barrier', '.LBB')) or 's_cbranch' in l:
        out.append(l.split(';')[0][:70])
print(n, len(body), 'lines')
print('\n'.join(out[:lim]))
for key in ('vgpr_count', 'sgpr_count', 'scratch', 'NumVgprs', 'ScratchSize', 'Occupancy'):
    for l in s[j:j + 4000].split('\n'):
        if key in l:
            print(l.strip())
            break
