# Audit of gemm.hip's inline-asm weight loads in the dequant-fused GEMM (guide §5.7 item 1): no instruction may
# touch an asm load's destination registers between the load and the wait that names them.
# Usage: hipcc ... -save-temps -c csrc/kernels/gemm.hip in /tmp/isa, then python tools/audit_asm_loads.py
import re,sys
s=open('/tmp/isa/gemm-hip-amdgcn-amd-amdhsa-gfx950.s').read()
def regs_of(l):
    used=set()
    for a,b,c in re.findall(r'v\[(\d+):(\d+)\]|v(\d+)',l.split(';')[0]):
        if c: used.add(int(c))
        else: used.update(range(int(a),int(b)+1))
    return used
bad=0
for name in re.findall(r'^(_ZN5acemi12_GLOBAL__N_113gemm_q_kernel[A-Za-z0-9_]*):', s, re.M):
    i=s.index(name+':'); j=s.index('.Lfunc_end',i); body=[l.strip() for l in s[i:j].splitlines()]
    labels={l.split()[0].rstrip(':'):k for k,l in enumerate(body) if l.startswith('.LBB')}
    top=None
    for k,l in enumerate(body):
        m=re.match(r's_cbranch_scc[01] (\.LBB\d+_\d+)',l)
        if m and labels.get(m.group(1),1e9)<k: top=labels[m.group(1)]; bot=k; break
    loop=[l for l in body[top:bot+1] if l and not l.startswith(';')]
    # wait_wq = first 's_waitcnt vmcnt' after the last ds_read_b128 of the loop top
    lastread=max(k for k,l in enumerate(loop) if l.startswith('ds_read_b128'))
    wq=next(k for k in range(lastread,len(loop)) if loop[k].startswith('s_waitcnt vmcnt'))
    for k,l in enumerate(loop):
        if not re.match(r'global_load_dword(x2|x4)? ',l): continue
        dest=regs_of(l.split(',')[0])
        seq=loop[k+1:]+loop[:wq]
        for l2 in seq:
            if regs_of(l2)&dest and not l2.startswith('global_load_dword'):
                bad+=1; print(name[-45:], l, '->', l2); break
print('kernels checked; bad =', bad)
bad=0
for name in re.findall(r'^(_ZN5acemi12_GLOBAL__N_113gemm_q_kernel[A-Za-z0-9_]*):', s, re.M):
    i=s.index(name+':'); j=s.index('.Lfunc_end',i); body=[l.strip() for l in s[i:j].splitlines()]
    labels={l.split()[0].rstrip(':'):k for k,l in enumerate(body) if l.startswith('.LBB')}
    for k,l in enumerate(body):
        m=re.match(r's_cbranch_scc[01] (\.LBB\d+_\d+)',l)
        if m and labels.get(m.group(1),1e9)<k: top=labels[m.group(1)]; break
    pro=[l for l in body[:top] if l and not l.startswith(';')]
    for k,l in enumerate(pro):
        if not re.match(r'global_load_dword(x2|x4)? ',l): continue
        dest=regs_of(l.split(',')[0])
        for l2 in pro[k+1:]:
            if l2.startswith('s_waitcnt vmcnt'): break
            if regs_of(l2)&dest and not l2.startswith('global_load_dword'):
                bad+=1; print('PROLOGUE', name[-45:], l, '->', l2); break
print('prologue bad =', bad)
