"""hipGraph capture/replay for fixed launch sequences (torch.cuda.CUDAGraph is hipGraph on ROCm).

The framework's native launchers enqueue on torch's current stream, so a sequence of them (and
of small torch ops on preallocated buffers) records into a graph unchanged.  Capture never
executes the work: run the sequence once eagerly first when its side effects matter.
"""
from __future__ import annotations

import logging

import torch

logger = logging.getLogger(__name__)


class Graph:
    def __init__(self, g: torch.cuda.CUDAGraph):
        self.g = g

    def replay(self):
        self.g.replay()


def capture(fn, pool=None) -> "Graph | None":
    """Record ``fn()`` into a hipGraph on a side stream; None (caller stays eager) on failure."""
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    try:
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, pool=pool, stream=s):
                fn()
    except Exception as e:  # noqa: BLE001 - capture is an optimisation
        logger.warning("hipGraph capture failed (%s); running eagerly", e)
        torch.cuda.current_stream().wait_stream(s)
        return None
    torch.cuda.current_stream().wait_stream(s)
    return Graph(g)
