"""Host thread pool (``DL/utils/ThreadPool.scala:38-270``): ``invokeAndWait``, ``invokeAndWait2``
(timeout: unfinished tasks are cancelled and reported — the straggler-dropping primitive),
``invoke`` and ``sync``.  Device work goes to HIP streams; this pool serves host-side work
(data loading, decode, checkpoint writing)."""
from __future__ import annotations

import concurrent.futures as cf
from typing import Callable, List, Optional, Sequence


class ThreadPool:
    def __init__(self, pool_size: int = 4):
        self.poolSize = max(1, int(pool_size))
        self._ex = cf.ThreadPoolExecutor(max_workers=self.poolSize)

    def getPoolSize(self) -> int:
        return self.poolSize

    def invokeAndWait(self, tasks: Sequence[Callable], timeout: Optional[float] = None) -> List:
        futs = [self._ex.submit(t) for t in tasks]
        return [f.result(timeout=timeout) for f in futs]

    def invokeAndWait2(self, tasks: Sequence[Callable], timeout: Optional[float] = None) -> List[cf.Future]:
        """Run ``tasks``; after ``timeout`` seconds the unfinished ones are cancelled.  Returns the
        futures (``f.done()`` / ``f.cancelled()`` tell which finished)."""
        futs = [self._ex.submit(t) for t in tasks]
        done, pending = cf.wait(futs, timeout=timeout)
        for f in pending:
            f.cancel()
        return futs

    def invoke(self, task: Callable) -> cf.Future:
        return self._ex.submit(task)

    def invoke_all(self, tasks: Sequence[Callable]) -> List[cf.Future]:
        return [self._ex.submit(t) for t in tasks]

    def sync(self, futures: Sequence[cf.Future], timeout: Optional[float] = None):
        for f in futures:
            f.result(timeout=timeout)

    def shutdown(self):
        self._ex.shutdown(wait=True)

    # MKL thread knobs are host-BLAS concerns; accepted for API parity
    def setMKLThread(self, size: int):
        import torch
        torch.set_num_threads(max(1, int(size)))
        return self
