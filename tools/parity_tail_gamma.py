"""Per-tensor gradient cosine of one ResNet-50 bf16 step vs the fp32 host oracle at several block-tail
γ values, native HIP path vs torch bf16 ops (run on a GPU: python tools/parity_tail_gamma.py)."""
import sys; sys.path.insert(0, "tests"); sys.path.insert(0, "bigdl-1_amd")
import test_train_parity as t
t._setup_bf16()
for g in (0.1, 0.25):
    for nat in (True, False):
        lg, lc, cos = t._grad_cosines(50, native=nat, tail_gamma=g)
        cs = sorted(cos)
        print(f"gamma {g} native {nat}: loss {lg:.5f}/{lc:.5f} min {cs[0]:.4f} p10 {cs[len(cs)//10]:.4f} med {cs[len(cs)//2]:.4f}", flush=True)
