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


class NativeGraph:
    """A hipGraph captured and launched through the native extension (hipStreamBeginCapture in
    thread-local mode / hipGraphInstantiate / hipGraphLaunch) rather than torch.cuda.CUDAGraph,
    whose replay() waited for the device on this build (profiles/r6_j: a DP SGD replay call cost
    the fit's whole device time on the host).  Capture records the caller's launches on a side
    stream made torch's current stream; replay launches on the current stream."""

    def __init__(self, exec_handle: int):
        self.h = int(exec_handle)

    def replay(self):
        from ..ops.native import native

        native().graph_launch(self.h, torch.cuda.current_stream().cuda_stream)

    def __del__(self):
        try:
            from ..ops.native import native

            native().graph_destroy(self.h)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def capture_native(fn) -> "NativeGraph | None":
    """Record ``fn()`` (which launches on torch's current stream) into a native hipGraph; None on
    failure (the caller stays eager).  Like capture(), nothing executes during capture."""
    from ..ops.native import native

    m = native()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    began = False
    try:
        with torch.cuda.stream(s):
            m.graph_begin(s.cuda_stream)
            began = True
            fn()
            h = m.graph_end(s.cuda_stream)
            began = False
    except Exception as e:  # noqa: BLE001 - capture is an optimisation
        if began:
            try:
                m.graph_destroy(m.graph_end(s.cuda_stream))
            except Exception:  # noqa: BLE001
                pass
        logger.warning("native hipGraph capture failed (%s); running eagerly", e)
        torch.cuda.current_stream().wait_stream(s)
        return None
    torch.cuda.current_stream().wait_stream(s)
    return NativeGraph(h)
