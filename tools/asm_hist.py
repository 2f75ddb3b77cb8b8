"""Instruction histogram of one kernel in a hipcc -S dump: python tools/asm_hist.py file.s substring"""
import sys
from collections import Counter

s = open(sys.argv[1]).read().splitlines()
start = next(i for i, l in enumerate(s) if sys.argv[2] in l and l.split(';')[0].rstrip().endswith(':') and not l.startswith('\t'))
end = next(i for i in range(start, len(s)) if 's_endpgm' in s[i])
c = Counter(l.split()[0] for l in s[start:end] if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'))
print(end - start, 'lines')
print(sorted(c.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30])
