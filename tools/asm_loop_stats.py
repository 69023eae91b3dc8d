#!/usr/bin/env python3
"""Instruction mix of the innermost loop around a pattern in a hipcc --save-temps .s file.

    python tools/asm_loop_stats.py <file.s> <kernel-symbol-substring> <regex> [nth]
Counts VALU / SALU / branch / LDS / VMEM instructions in the blocks of that loop (nested
child loops excluded), i.e. the straight-line cost of one iteration.
"""
import re
import sys


def main():
    path, ksub, pat = sys.argv[1:4]
    nth = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    L = open(path).read().split('\n')
    start = next(i for i, l in enumerate(L) if re.match(r'^\S*' + re.escape(ksub) + r'\S*:', l) or (ksub in l and l.endswith(':') and not l.startswith('\t')))
    end = next(i for i in range(start, len(L)) if 's_endpgm' in L[i])
    K = L[start:end]
    hits = [i for i, l in enumerate(K) if re.search(pat, l)]
    h = hits[nth]
    # loop header of the block containing h: walk back to the nearest label, read its "Loop: Header=" note
    blk = max(i for i in range(h + 1) if re.match(r'^(\.LBB\S+:|; %bb)', K[i]))
    hdr = None
    for i in range(blk, min(blk + 4, len(K))):
        m = re.search(r'Header=(BB\S+) Depth=(\d+)', K[i])
        if m:
            hdr, depth = m.group(1), int(m.group(2))
            break
    if hdr is None:
        m = re.match(r'^\.L(BB\S+):', K[blk])
        hdr, depth = m.group(1), 1
    # blocks belonging to this loop at this depth
    counts = dict(valu=0, salu=0, branch=0, lds=0, vmem=0, wait=0)
    blocks = 0
    cur_in = False
    for i, l in enumerate(K):
        if re.match(r'^(\.LBB\S+:|; %bb)', l):
            note = ' '.join(K[i:i + 3])
            m = re.search(r'Header=(BB\S+) Depth=(\d+)', note)
            cur_in = bool(m and m.group(1) == hdr and int(m.group(2)) == depth) or l.startswith('.L' + hdr + ':')
            blocks += cur_in
            continue
        if not cur_in:
            continue
        t = l.strip()
        if t.startswith('s_cbranch') or t.startswith('s_branch'):
            counts['branch'] += 1
        elif t.startswith('s_waitcnt'):
            counts['wait'] += 1
        elif t.startswith('ds_'):
            counts['lds'] += 1
        elif t.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
            counts['vmem'] += 1
        elif t.startswith('v_'):
            counts['valu'] += 1
        elif t.startswith('s_'):
            counts['salu'] += 1
    print(f"loop {hdr} depth {depth}: {blocks} blocks", counts)


if __name__ == '__main__':
    main()
