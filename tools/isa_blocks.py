"""Per-basic-block instruction mix of one kernel in a gfx950 .s file (VALU / SALU / LDS / VMEM /
MFMA); the blocks holding MFMAs are the hot loop.  Usage: python tools/isa_blocks.py FILE.s KERNEL"""
import re
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"^(_ZN[^\s:]*%s[^\s:]*):" % re.escape(kern), s, re.M)
    start = m.end()
    end = s.find('.Lfunc_end', start)
    body = s[start:end].splitlines()
    blocks, cur, name = [], [], 'entry'
    for ln in body:
        t = ln.strip()
        if re.match(r'^\.LBB\d+_\d+:', t):
            blocks.append((name, cur))
            name, cur = t[:-1], []
            continue
        if not t or t.startswith(';') or t.startswith('.'):
            continue
        cur.append(t.split()[0])
    blocks.append((name, cur))
    tot = {}
    for name, ins in blocks:
        c = {'valu': 0, 'salu': 0, 'lds': 0, 'vmem': 0, 'mfma': 0, 'other': 0}
        for op in ins:
            if op.startswith('v_mfma'):
                c['mfma'] += 1
            elif op.startswith('v_'):
                c['valu'] += 1
            elif op.startswith('s_'):
                c['salu'] += 1
            elif op.startswith('ds_'):
                c['lds'] += 1
            elif op.startswith(('global_', 'buffer_', 'flat_')):
                c['vmem'] += 1
            else:
                c['other'] += 1
        if c['mfma'] or '-a' in sys.argv:
            print(name, len(ins), c)
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
    print('total', tot)


if __name__ == '__main__':
    main()
