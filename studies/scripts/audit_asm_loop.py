"""Audit an asm-scheduled kernel's main loop in a hipcc -save-temps .s: print every instruction the COMPILER
emitted (outside ;;#ASMSTART/;;#ASMEND) between the first and last MFMA of the kernel, so register copies or
waits that could read an asynchronously written register are visible.  usage: audit_asm_loop.py file.s symbol"""
import sys

s = open(sys.argv[1]).read()
sym = sys.argv[2]
k = s[s.index(sym + ':'):]
k = k[:k.index('.Lfunc_end')]
lines = k.split('\n')
inasm = False
outside = []
for i, l in enumerate(lines):
    t = l.strip()
    if t.startswith(';;#ASMSTART'):
        inasm = True
        continue
    if t.startswith(';;#ASMEND'):
        inasm = False
        continue
    if not inasm and t and not t.startswith(';') and not (t.startswith('.') and not t.startswith('.LBB')):
        outside.append((i, t))
mf = [i for i, l in enumerate(lines) if 'v_mfma' in l]
print('mfma statements', len(mf), 'lines', mf[0], '..', mf[-1])
for i, t in outside:
    if mf[0] - 40 < i < mf[-1] + 10:
        print(i, t)
