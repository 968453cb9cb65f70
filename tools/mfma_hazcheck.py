"""Static check of the inline-asm MFMAs in fatchord_xcdm.hip (hipcc does not pad hazards around
inline asm): no VALU write to an MFMA source within 2 wait states before it, no non-MFMA read of
an MFMA result within 8 (4x4x1) / 19 (16x16x4) wait states after it.  Input: the device asm,
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -fno-slp-vectorize --cuda-device-only -S \
        -o /tmp/xcdm.s wavernn_amd/csrc/fatchord_xcdm.hip"""
import re,sys
s=open('/tmp/xcdm.s').read()
def regs(tok):
    # expand v5 / v[4:7] / a3 / a[0:3]
    out=set()
    for m in re.finditer(r'([va])\[(\d+):(\d+)\]|([va])(\d+)\b',tok):
        if m.group(1): out|={m.group(1)+str(i) for i in range(int(m.group(2)),int(m.group(3))+1)}
        else: out.add(m.group(4)+m.group(5))
    return out
for nq in '1234':
    a=s.index('_ZN4wrnn20fatchord_xcdm_kernelILi%sELb0EEEvNS_8XcdmArgsE: ;'%nq)
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
                        print("NQ",nq,"VALU->MFMA hazard:",p,"|",l); bad+=1
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
                        print("NQ",nq,"MFMA->read hazard:",l,"|",p,"ws",ws); bad+=1
                ws+=1; j+=1
    print("NQ",nq,"mfma",sum(1 for l in ins if l.startswith('v_mfma')),"hazards",bad)
