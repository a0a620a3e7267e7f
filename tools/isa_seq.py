"""Compress a kernel's gfx950 ISA (hipcc --save-temps .s) into an instruction-class
sequence: L/S global load/store, w/r LDS write/read, B barrier, |waitcnt|,
X scratch, J branch, '.' VALU runs.  usage: isa_seq.py file.s name-substring"""
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
m = [mm for mm in re.finditer(r'^(_Z\S+):', s, re.M) if key in mm.group(1)][0]
start = m.end()
end = s.index('.Lfunc_end', start)
seq = []
for ln in s[start:end].split('\n'):
    t = ln.strip()
    if not t or t[0] in ';.' or t.endswith(':'):
        if t.endswith(':') and t.startswith('.LBB'):
            seq.append('\n' + t + ' ')
        continue
    op = t.split()[0]
    if op.startswith(('global_load', 'buffer_load')): c = 'L'
    elif op.startswith(('global_store', 'buffer_store')): c = 'S'
    elif op.startswith('ds_write'): c = 'w'
    elif op.startswith('ds_read'): c = 'r'
    elif op.startswith('s_waitcnt'): c = '|' + t.split(None, 1)[1].replace(' ', '') + '|'
    elif op == 's_barrier': c = 'B'
    elif op.startswith('v_'): c = '.'
    elif op.startswith('scratch'): c = 'X'
    elif op.startswith(('s_cbranch', 's_branch')): c = 'J'
    else: c = ''
    seq.append(c)
out = ''.join(seq)
out = re.sub(r'\.{6,}', lambda q: '.{%d}' % len(q.group(0)), out)
print(m.group(1)[:60])
print(out)
