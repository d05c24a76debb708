import sys, time, torch
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "bigdl-1_amd"))
from bigdl.ops import native
def t(f, n=50):
    for _ in range(5): f()
    torch.cuda.synchronize(); a = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter() - a) / n * 1e3
for rows, H in [(8192, 512), (16384, 1024), (4096, 4096)]:
    x = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(H, device="cuda", requires_grad=True); b = torch.zeros(H, device="cuda", requires_grad=True)
    gy = torch.randn_like(x)
    def nat():
        native.layer_norm(x, w, b, 1e-6).backward(gy)
    def comp():
        mu = x.mean(-1, keepdim=True); var = ((x - mu) ** 2).mean(-1, keepdim=True)
        ((x - mu) * torch.rsqrt(var + 1e-6) * w.to(x.dtype) + b.to(x.dtype)).backward(gy)
    def tl():
        torch.nn.functional.layer_norm(x, (H,), w.to(x.dtype), b.to(x.dtype), 1e-6).backward(gy)
    fwd = t(lambda: native.layer_norm(x.detach(), w.detach(), b.detach(), 1e-6))
    gb = rows * H * 2 * 2 / 1e9
    print(f"rows={rows} H={H} native_fwd={fwd:.4f}ms ({gb/fwd:.2f} TB/s) native_fb={t(nat):.4f}ms composed_fb={t(comp):.4f}ms torch_ln_fb={t(tl):.4f}ms", flush=True)
