"""Instruction mix per basic block of one kernel in a hipcc -S listing (gfx950).

usage: python scripts/tools/isa_count.py <file.s> <kernel-name-substring> [min_insts]

Prints, per basic block of the kernel (in listing order, blocks of >= min_insts instructions):
label, VALU (v_*; v_pk_* counted separately too), LDS (ds_*), SALU (s_*), VMEM (global_/buffer_)
and s_waitcnt counts, plus the branch that ends it — enough to find the pass loop and compare
builds (the profile's per-frame VALU count is per pass / 4 frames).
"""
import re
import sys


def main():
    path, want = sys.argv[1], sys.argv[2]
    min_insts = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    s = open(path).read()
    names = [n for n in re.findall(r'^(\S+):\s*(?:;.*)?$', s, re.M) if want in n and not n.startswith('.')]
    if not names:
        sys.exit(f"no kernel matching {want}")
    name = names[0]
    a = s.index(name + ':')
    b = s.index('.Lfunc_end', a)
    blocks, cur, label = [], [], name
    for line in s[a:b].splitlines()[1:]:
        t = line.strip()
        if not t or t.startswith(';') or t.startswith('.'):
            if re.match(r'^\.LBB\S*:', t):
                blocks.append((label, cur))
                label, cur = t.rstrip(':').split()[0].rstrip(':'), []
            continue
        if re.match(r'^\S+:', t):
            continue
        cur.append(t.split(';')[0].strip())
    blocks.append((label, cur))
    tot = dict(valu=0, pk=0, lds=0, salu=0, vmem=0)
    print(f"{name}\n{'block':<14}{'n':>6}{'VALU':>6}{'pk':>5}{'LDS':>5}{'SALU':>6}{'VMEM':>6}{'wait':>6}  end")
    for lab, ins in blocks:
        ops = [i.split()[0] for i in ins if i]
        valu = sum(o.startswith('v_') for o in ops)
        pk = sum(o.startswith('v_pk_') for o in ops)
        lds = sum(o.startswith('ds_') for o in ops)
        salu = sum(o.startswith('s_') and not o.startswith('s_waitcnt') for o in ops)
        vmem = sum(o.startswith(('global_', 'buffer_')) for o in ops)
        wait = sum(o.startswith('s_waitcnt') for o in ops)
        for k, v in zip(tot, (valu, pk, lds, salu, vmem)):
            tot[k] += v
        if len(ops) >= min_insts:
            end = next((i for i in reversed(ins) if i.startswith('s_cbranch') or i.startswith('s_branch')), '')
            print(f"{lab:<14}{len(ops):>6}{valu:>6}{pk:>5}{lds:>5}{salu:>6}{vmem:>6}{wait:>6}  {end}")
    print('total', tot)


if __name__ == '__main__':
    main()
