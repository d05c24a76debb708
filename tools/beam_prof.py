"""Transformer translation with beam search on the GPU (the workload of ``SequenceBeamSearch``,
``DL/nn/SequenceBeamSearch.scala:37``, driving ``Attention.updateOutputCache``,
``DL/nn/Attention.scala:118-140``): runs a few decodes so a ``rocprofv3 --kernel-trace --stats`` of
this script shows which attention kernels the cached decoding launches.  Prints one JSON line with
the decode time and the torch-fallback counters."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd"))


def main():
    import torch
    from bigdl.ops import fallback_counts, reset_fallbacks
    from bigdl.nn.layers.attention import Transformer, SequenceBeamSearch
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    V, H, heads, filt, layers = 1000, 512, 8, 2048, 2
    B, L, beam, max_dec = 8, 32, 4, 32
    bs = SequenceBeamSearch(V, beam, 0.6, max_dec, 3, 0, 2, H)
    tr = Transformer(V, H, heads, filt, layers, 1.0, 1.0, 1.0, with_share_weights_linear=True,
                     transformer_type="Translation", beam_search=bs)
    tr.evaluate()
    tr = tr.cuda()
    src = torch.randint(3, V, (B, L), device="cuda").float()
    with torch.no_grad():
        tr.forward(src)  # warm-up
        torch.cuda.synchronize()
        reset_fallbacks()
        t0 = time.perf_counter()
        n = 3
        for _ in range(n):
            tr.forward(src)
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    print(json.dumps({"workload": "transformer_beam_search", "batch": B, "src_len": L, "beam": beam,
                      "hidden": H, "heads": heads, "layers": layers, "max_decode": max_dec,
                      "ms_per_decode": round(ms, 2), "fallbacks": fallback_counts()}), flush=True)


if __name__ == "__main__":
    main()
