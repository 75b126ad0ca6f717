"""fp32 GEMM calibration of the box: torch.matmul (hipBLASLt/rocBLAS, exact fp32) at several shapes."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
def t(m, n, k, it=20):
    a = torch.randn(m, k, device="cuda"); b = torch.randn(k, n, device="cuda")
    for _ in range(3): a @ b
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): a @ b
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / it
    print(f"{m}x{n}x{k}: {2*m*n*k/ms/1e9:.1f} TF/s ({ms*1e3:.1f} us)", flush=True)
for shp in [(8192, 8192, 8192), (4096, 4096, 4096), (64, 119808, 576), (128, 29952, 1152), (256, 7488, 2304), (512, 1872, 4608)]:
    t(*shp)
