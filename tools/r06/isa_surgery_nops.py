import re, subprocess, sys
src = open(sys.argv[1]).read().split('\n')
mode, out = sys.argv[2], sys.argv[3]
res = []
in_render = False
for ln in src:
    if ln.startswith('rt_accel_render:'): in_render = True
    elif re.match(r'^rt_accel_render_count:', ln): in_render = False
    res.append(ln)
    if not in_render: continue
    t = ln.strip()
    if mode == 'readlane' and t.startswith('v_readlane_b32'): res.append('\ts_nop 4')
    if mode == 'writelane' and t.startswith('v_writelane_b32'): res.append('\ts_nop 4')
    if mode == 'both' and (t.startswith('v_readlane_b32') or t.startswith('v_writelane_b32')): res.append('\ts_nop 4')
open(out + '.s', 'w').write('\n'.join(res))
L = '/opt/rocm/lib/llvm/bin'
subprocess.run([f'{L}/clang', '-x', 'assembler', '-target', 'amdgcn-amd-amdhsa', '-mcpu=gfx950', '-c', out + '.s', '-o', out + '.o'], check=True)
subprocess.run([f'{L}/ld.lld', '-shared', out + '.o', '-o', out + '.co'], check=True)
print(out, 'ok')
