"""register / scratch use of each kernel in a hipcc -save-temps .s file, and the instruction mix of one"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r'\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel', s, re.S):
    body = m.group(2)
    g = lambda k: re.search(r'\.amdhsa_' + k + r'\s+(\S+)', body).group(1)
    print(m.group(1)[:70], 'vgpr', g('next_free_vgpr'), 'sgpr', g('next_free_sgpr'), 'scratch', g('private_segment_fixed_size'))
if len(sys.argv) > 2:
    a = re.search('^' + re.escape(sys.argv[2]) + ':', s, re.M).start()
    b = s.index('s_endpgm', a)
    L = [l.strip() for l in s[a:b].split('\n')]
    ins = [l for l in L if l and not l.startswith(('.', ';')) and not l.endswith(':') and not l.startswith('_Z')]
    print('instructions', len(ins))
    c = collections.Counter(l.split()[0] for l in ins)
    print(' '.join(f'{k}:{v}' for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30)))
