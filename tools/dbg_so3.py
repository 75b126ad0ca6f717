import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch, md2hip
from md2hip._lib import check, lib, ptr, stream_of
from tests import _data as D
N = 5
poses = D.poses(N, seed=3)
pose = md2hip.pack_poses([(r.float(), t.float()) for r, t in poses]).cuda()
print(pose.shape, pose.dtype, pose.is_contiguous())
Rt = torch.zeros(2 * N, 12, device="cuda")
rc = lib().md2_so3_compose_fwd(ptr(pose), N, 1, ptr(Rt), stream_of())
print("rc", rc, lib().md2_last_error())
torch.cuda.synchronize()
print(Rt[:2])
