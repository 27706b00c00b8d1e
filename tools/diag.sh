cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
{
env | grep -i -E "HIP|ROCR|CUDA|GPU|HSA" ;
ls -la /dev/kfd /dev/dri 2>&1 | head;
timeout 60 rocminfo 2>&1 | grep -E "Name:|Marketing" | head -8;
timeout 120 python -c "
import ctypes, sys
sys.path.insert(0,'pt-bpe_amd')
from geobpe import _native
L=_native.lib()
c=ctypes.c_void_p()
rc=L.geobpe_create(ctypes.byref(c),0,None,1000)
print('create without torch rc',rc, L.geobpe_last_error(c))
";
timeout 120 python -c "
import torch; print('torch avail', torch.cuda.is_available(), torch.cuda.device_count())
import ctypes, sys
sys.path.insert(0,'pt-bpe_amd')
from geobpe import _native
L=_native.lib()
c=ctypes.c_void_p()
rc=L.geobpe_create(ctypes.byref(c),0,None,1000)
print('create after torch rc',rc, L.geobpe_last_error(c))
";
} > gpurun_out/diag.log 2>&1
