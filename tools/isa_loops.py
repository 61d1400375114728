# Loops of a disassembled kernel (tools/isa_one.sh): size, VALU, LDS, scratch, AGPR moves, DPP per loop
#   python3 tools/isa_loops.py out.s [min_len] [max_len]
import re,sys
lines=open(sys.argv[1]).read().split('\n')
ins=[]
for l in lines:
    m=re.match(r'\s+(\S+.*?)\s*//\s*([0-9A-F]+):',l)
    if m: ins.append((int(m.group(2),16),m.group(1)))
idx={a:k for k,(a,t) in enumerate(ins)}
minlen=int(sys.argv[2]) if len(sys.argv)>2 else 100
maxlen=int(sys.argv[3]) if len(sys.argv)>3 else 1000
for k,(a,t) in enumerate(ins):
    m=re.match(r'(s_cbranch_\w+|s_branch)\s+(-?\d+)',t)
    if not m: continue
    s=int(m.group(2)); s = s-65536 if s>=32768 else s
    if s>=0: continue
    j=idx.get(a+4+s*4)
    if j is None or not (minlen<=k-j+1<=maxlen): continue
    body=[x for _,x in ins[j:k+1]]
    c=lambda p: sum(1 for x in body if x.startswith(p))
    print(f"{j:6d}-{k:6d} n={len(body):4d} v={c('v_'):4d} ds={c('ds_'):3d} scr={c('scratch_')+c('buffer_'):3d} acc={c('v_accvgpr'):3d} nop={c('s_nop'):3d} dpp={sum(1 for x in body if 'quad_perm' in x or 'row_' in x):3d} cnd={c('v_cndmask'):3d} rl={c('v_readlane'):3d}")
