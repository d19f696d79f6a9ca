import re, subprocess, sys
src = open(sys.argv[1]).read().split('\n')
out = sys.argv[2]
# move the exec restore of .LBB0_164 (%.loopexit.i.i, rt_accel_render) above the split copies placed before it
i = src.index('.LBB0_164:                              ; %.loopexit.i.i')
j = next(k for k in range(i, i + 40) if src[k].strip().startswith('s_or_b64 exec, exec, s[10:11]'))
print('copies moved:', [s.strip() for s in src[i + 2:j]])
line = src.pop(j)
src.insert(i + 2, line)
open(out + '.s', 'w').write('\n'.join(src))
L = '/opt/rocm/lib/llvm/bin'
subprocess.run([f'{L}/clang', '-x', 'assembler', '-target', 'amdgcn-amd-amdhsa', '-mcpu=gfx950', '-c', out + '.s', '-o', out + '.o'], check=True)
subprocess.run([f'{L}/ld.lld', '-shared', out + '.o', '-o', out + '.co'], check=True)
