"""Per-step wall times of the fp32 ResNet-50 training step (outlier hunt): bench.py's model / optimizer,
a device synchronize after every step, and the caching allocator's retry / malloc counters."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "bigdl-1_amd"))
import torch
import bench
from bigdl.utils import config
from bigdl.utils.engine import Engine

args = bench._parse(["--dtype", os.environ.get("DT", "fp32"), "--steps", "1"])
config.set_property("bigdl.compute.dtype", args.dtype)
config.set_property("bigdl.comm.dtype", "fp32")
Engine.init(dist=False)
dev = torch.device("cuda")
from bigdl.optim.optimizer import LocalOptimizer
model, crit, sgd, batches = bench._build(args, dev, 0)
opt = LocalOptimizer(model, [batches[0]], crit, sgd, batch_size=args.batch)
opt.prepare()
for i in range(int(os.environ.get("STEPS", "16"))):
    st = torch.cuda.memory_stats()
    t0 = time.perf_counter()
    opt.train_step(batches[i % 2])
    t1 = time.perf_counter()
    if os.environ.get("SYNC", "1") == "1" or i < 4:
        torch.cuda.synchronize()
    t2 = time.perf_counter()
    st2 = torch.cuda.memory_stats()
    print(f"step {i}: host {1e3 * (t1 - t0):8.2f} ms  total {1e3 * (t2 - t0):8.2f} ms  "
          f"mallocs +{st2.get('num_device_alloc', 0) - st.get('num_device_alloc', 0)} "
          f"retries +{st2.get('num_alloc_retries', 0) - st.get('num_alloc_retries', 0)} "
          f"overlap={getattr(opt, '_overlap_now', None)}", flush=True)
t0 = time.perf_counter()
torch.cuda.synchronize()
print(f"final drain {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
