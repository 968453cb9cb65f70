"""Static check of the inline-asm MFMAs in fatchord_xcdm.hip (MoL and RAW heads) and deepmind_xcd.hip (hipcc does not
pad hazards around inline asm): no VALU write to an MFMA source within 2 wait states before it,
no non-MFMA read of an MFMA result within 8 (4x4x1) / 19 (16x16x4) wait states after it.
Compiles the device asm of both files itself (hipcc, gfx950) into /tmp.

    python tools/mfma_hazcheck.py"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = [("fatchord_xcdm.hip", ["_ZN4wrnn20fatchord_xcdm_kernelILi%sELb0ELb%dEEEvNS_8XcdmArgsE" % (q, raw)
                                   for q in "1234" for raw in (0, 1)]),
           ("deepmind_xcd.hip", ["_ZN4wrnn19deepmind_xcd_kernelILb0EEEvNS_6DxArgsE"])]
def regs(tok):
    # expand v5 / v[4:7] / a3 / a[0:3]
    out=set()
    for m in re.finditer(r'([va])\[(\d+):(\d+)\]|([va])(\d+)\b',tok):
        if m.group(1): out|={m.group(1)+str(i) for i in range(int(m.group(2)),int(m.group(3))+1)}
        else: out.add(m.group(4)+m.group(5))
    return out
def asm(src):
    out = "/tmp/hazcheck_" + src.replace(".hip", ".s")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(REPO, "include"),
                    "-fno-slp-vectorize", "--cuda-device-only", "-S", "-o", out,
                    os.path.join(REPO, "wavernn_amd", "csrc", src)], check=True, capture_output=True)
    return open(out).read()
total = 0
for src, syms in KERNELS:
  s = asm(src)
  for sym in syms:
    nq = sym
    a=s.index(sym + ':')
    b=s.index('.Lfunc_end',a)
    ins=[l.strip() for l in s[a:b].split('\n')]
    ins=[l for l in ins if l and not l.startswith(';') and not l.startswith('.') and not l.endswith(':')]
    bad=0
    for i,l in enumerate(ins):
        if l.startswith('v_mfma'):
            ops=l.split(None,1)[1].split(',')
            dst=regs(ops[0]); srcab=regs(ops[1])|regs(ops[2]); srcc=regs(ops[3]) if len(ops)>3 else set()
            # look back: VALU writes within 2 wait states (count instrs, s_nop n counts n+1)
            ws=0; j=i-1
            while j>=0 and ws<3:
                p=ins[j]
                if p.startswith('s_nop'):
                    ws+=int(p.split()[1])+1; j-=1; continue
                if p.startswith('v_') and not p.startswith('v_mfma'):
                    d=regs(p.split(None,1)[1].split(',')[0]) if ' ' in p else set()
                    if d & (srcab|srcc):
                        print(sym,"VALU->MFMA hazard:",p,"|",l); bad+=1
                ws+=1; j-=1
            # look ahead: non-MFMA reading dst within 8 wait states
            ws=0; j=i+1
            while j<len(ins) and ws<(19 if '16x16' in l else 8):
                p=ins[j]
                if p.startswith('s_nop'):
                    ws+=int(p.split()[1])+1; j+=1; continue
                if not p.startswith('v_mfma') and (p.startswith('v_') or p.startswith('ds_') or p.startswith('global_') or p.startswith('buffer_')):
                    srcs=set()
                    parts=p.split(None,1)
                    if len(parts)>1:
                        ops2=parts[1].split(',')
                        srcs=set().union(*[regs(o) for o in ops2])
                    if srcs & dst:
                        print(sym,"MFMA->read hazard:",l,"|",p,"ws",ws); bad+=1
                ws+=1; j+=1
    print(src, sym, "mfma", sum(1 for l in ins if l.startswith('v_mfma')), "hazards", bad)
    total += bad
sys.exit(1 if total else 0)
