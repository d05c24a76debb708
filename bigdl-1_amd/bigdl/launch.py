"""Multi-GPU launcher: one process per GPU on one node (the role of the reference's
``scripts/spark-submit-with-bigdl.sh`` + Spark executors, SURVEY §2.13 CLI row).

    python -m bigdl.launch --nproc 8 train.py --arg ...
    python -m bigdl.launch --nproc 8 -m bigdl.models.train.imagenet --folder /data/imagenet-seq ...

Each rank gets ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``MASTER_ADDR`` / ``MASTER_PORT`` (the
``torch.distributed`` env:// contract that :class:`bigdl.utils.engine.Engine` reads; device =
``cuda:LOCAL_RANK``), is pinned to the CPU cores of its GPU's NUMA node (the reference pins its
parameter-sync threads, ``DistriParameterSynchronizer.scala:73,128-144``) and inherits the
RCCL/HIP environment.  Children are plain subprocesses started before anything touches the GPU;
the launcher waits for all of them, and if one fails it terminates the rest and returns its code.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gpu_numa_nodes() -> Dict[int, int]:
    """GPU index → NUMA node, from the DRM sysfs entries of AMD GPUs (render nodes in order)."""
    out: Dict[int, int] = {}
    base = "/sys/class/drm"
    try:
        cards = sorted((d for d in os.listdir(base) if d.startswith("renderD")), key=lambda d: int(d[7:]))
    except OSError:
        return out
    i = 0
    for c in cards:
        dev = os.path.join(base, c, "device")
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip() != "0x1002":
                    continue
            with open(os.path.join(dev, "numa_node")) as f:
                out[i] = max(0, int(f.read().strip()))
        except OSError:
            continue
        i += 1
    return out


def gpu_count() -> int:
    """Visible AMD GPUs without touching HIP: the DRM render nodes of vendor 0x1002, restricted by
    ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` when set."""
    n = len(gpu_numa_nodes())
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [t for t in v.split(",") if t.strip() != ""]
            n = min(n, len(ids)) if n else len(ids)
    return max(1, n)


def numa_cpus(node: int) -> Optional[List[int]]:
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
    except OSError:
        return None
    cpus: List[int] = []
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        elif part:
            cpus.append(int(part))
    return cpus or None


def rank_env(rank: int, world: int, addr: str, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR=addr, MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL / tensor sharing
    env.setdefault("OMP_NUM_THREADS", "4")
    return env


def launch(nproc: int, cmd: List[str], master_addr: str = "127.0.0.1", master_port: int = 0,
           bind_numa: bool = True, max_restarts: int = 0) -> int:
    """Run ``nproc`` ranks; if any rank fails, stop the others and relaunch ALL ranks (up to
    ``max_restarts`` times, SURVEY §5.3 supervisor).  ``BIGDL_RESTART_COUNT`` tells the script it is
    a restart (resume from the latest checkpoint, ``Optimizer`` does this when a checkpoint path is
    set)."""
    rc = 0
    for attempt in range(max_restarts + 1):
        os.environ["BIGDL_RESTART_COUNT"] = str(attempt)
        rc = _launch_once(nproc, cmd, master_addr, master_port, bind_numa)
        if rc in (0, 130):
            return rc
        print(f"[bigdl.launch] a rank failed with code {rc}; "
              f"{'restarting all ranks' if attempt < max_restarts else 'giving up'}", file=sys.stderr, flush=True)
    return rc


def _launch_once(nproc: int, cmd: List[str], master_addr: str, master_port: int, bind_numa: bool) -> int:
    port = master_port or _free_port()
    numa = gpu_numa_nodes() if bind_numa else {}
    procs = []
    for r in range(nproc):
        cpus = numa_cpus(numa[r]) if r in numa else None

        def pre(cpus=cpus):
            if cpus:
                try:
                    os.sched_setaffinity(0, cpus)
                except OSError:
                    pass
        procs.append(subprocess.Popen(cmd, env=rank_env(r, nproc, master_addr, port), preexec_fn=pre))
    rc = 0
    try:
        alive = list(procs)
        while alive:
            for p in list(alive):
                code = p.poll()
                if code is None:
                    continue
                alive.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in alive:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGINT)
        for p in procs:
            p.wait()
        return 130
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m bigdl.launch", description=__doc__.split("\n\n")[0])
    ap.add_argument("--nproc", "--nproc-per-node", dest="nproc", type=int, default=None,
                    help="processes (= GPUs) on this node; default: every visible GPU")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--no-numa-bind", action="store_true")
    ap.add_argument("--max-restarts", type=int, default=0, help="relaunch all ranks after a failure")
    ap.add_argument("-m", dest="module", default=None, help="run a module (python -m MODULE) instead of a script")
    ap.add_argument("script", nargs="?")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    argv = list(sys.argv[1:] if argv is None else argv)
    module_rest = None
    if "-m" in argv:  # everything after ``-m MODULE`` belongs to the module, like python -m
        i = argv.index("-m")
        if i + 1 >= len(argv):
            ap.error("-m needs a module name")
        module_rest = argv[i + 1:]
        argv = argv[:i]
    a = ap.parse_args(argv)
    if module_rest is not None:
        a.module, a.script, a.args = module_rest[0], None, module_rest[1:]
    if a.module is None and a.script is None:
        ap.error("a script or -m MODULE is required")
    n = a.nproc
    if n is None:
        n = gpu_count()  # sysfs only: the supervisor never loads the HIP runtime
    if a.module is not None:
        rest = ([a.script] if a.script is not None else []) + a.args
        cmd = [sys.executable, "-m", a.module] + rest
    else:
        cmd = [sys.executable, a.script] + a.args if a.script.endswith(".py") else [a.script] + a.args
    return launch(n, cmd, a.master_addr, a.master_port, not a.no_numa_bind, a.max_restarts)


if __name__ == "__main__":
    sys.exit(main())
