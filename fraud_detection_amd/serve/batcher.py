"""Async micro-batcher: coalesces concurrent /predict requests into one fused device launch.

The reference scores one row per request through pandas + sklearn (api/app.py:184-240) with no
batching.  On a GPU a single-row launch costs about as much as a thousand-row one, so requests
that arrive within ``window_us`` of each other share a launch (bounded by ``max_batch``).  The
launch runs on a worker thread so the event loop keeps accepting requests.  On CPU the window
defaults to 0 and requests run inline.
"""
from __future__ import annotations

import asyncio
import time

import numpy as np


class MicroBatcher:
    def __init__(self, engine, window_us: int = 300, max_batch: int = 4096, metrics=None):
        self.engine = engine
        self.window = max(0, window_us) / 1e6
        self.max_batch = max_batch
        self.metrics = metrics
        self._q: asyncio.Queue | None = None
        self._task: asyncio.Task | None = None

    @property
    def enabled(self) -> bool:
        return self.window > 0 and self.engine.device.type == "cuda"

    async def start(self):
        if self.enabled and self._task is None:
            self._q = asyncio.Queue()
            self._task = asyncio.create_task(self._run())

    async def stop(self):
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
            self._task = None

    async def submit(self, row: np.ndarray):
        """-> (prob, logit) for one row."""
        if not self.enabled or self._task is None:
            p, z = self.engine.predict_proba(row[None, :])
            self._observe(1)
            return float(p[0]), float(z[0])
        fut = asyncio.get_running_loop().create_future()
        await self._q.put((row, fut))
        return await fut

    def _observe(self, n):
        if self.metrics is not None:
            self.metrics.microbatch_size.observe(n)

    async def _run(self):
        loop = asyncio.get_running_loop()
        while True:
            row, fut = await self._q.get()
            rows, futs = [row], [fut]
            deadline = time.perf_counter() + self.window
            while len(rows) < self.max_batch:
                timeout = deadline - time.perf_counter()
                if timeout <= 0:
                    break
                try:
                    r, f = await asyncio.wait_for(self._q.get(), timeout)
                except asyncio.TimeoutError:
                    break
                rows.append(r)
                futs.append(f)
            X = np.stack(rows)
            try:
                p, z = await loop.run_in_executor(None, self.engine.predict_proba, X)
                self._observe(len(rows))
                for i, f in enumerate(futs):
                    if not f.done():
                        f.set_result((float(p[i]), float(z[i])))
            except Exception as e:  # noqa: BLE001
                for f in futs:
                    if not f.done():
                        f.set_exception(e)
