"""Collectives inside the training step, and HIP-graph capture around them.

The data-parallel step issues collectives in the middle of its forward / backward: the
contrastive loss's all_gather of the source codes (loss/contrast_loss.py) and, with SyncBN, the
per-layer statistics exchanges (ured_hip/syncbn.py). Every such call goes through run(). Eagerly
it just issues the collective. While engine/graph.py captures the step, run() instead closes
the captured segment, records the collective and opens the next segment: a replay is then
segment 0, collective 0, segment 1, ... — the collectives run eagerly between replays on
static buffers (no collective is captured into a graph, so the capture works with any
process-group backend, gloo included). With RCCL ("nccl"), whose collectives can be captured,
SegmentedCapture(inline=True) records them in the graph itself: one graph, no split, and the
bucketed gradient all-reduce issued from backward's hooks is captured with it (overlapping the
rest of the backward on RCCL's stream, engine/graph.py).
"""

_split = None
_active = None          # the SegmentedCapture being recorded (segmented or inline), else None


def capture_stream():
    """The stream the running segmented capture records on (None when nothing is captured)."""
    return None if _active is None else _active.stream


def run(fn):
    """Issue the collective `fn()` (no arguments, no return value; in- and outputs are tensors it
    closes over, at fixed addresses while a graph replays them)."""
    if _split is None:
        fn()
    else:
        _split(fn)


class SegmentedCapture:
    """Capture a region as a chain of HIP graphs split at run() calls (engine/graph.py).

        cap = SegmentedCapture(pool)
        with torch.cuda.stream(s):
            cap.begin(); <forward / backward>; cap.end()
        cap.replay()
    """

    def __init__(self, pool=None, inline=False):
        import torch
        self._torch = torch
        self.inline = inline
        self.pool = pool if pool is not None else torch.cuda.graph_pool_handle()
        self.graphs, self.collectives = [], []
        self._g = None

    def _open(self):
        # relaxed: a split inside backward closes the segment on the autograd engine's thread
        # and opens the next one there; the main thread closes the last one
        self._g = self._torch.cuda.CUDAGraph()
        self._g.capture_begin(pool=self.pool, capture_error_mode="relaxed")

    def _close(self):
        # two collectives with no kernel between them (e.g. the last gradient bucket's all-reduce
        # and the waits after the backward) leave an empty segment: valid, replays as a no-op
        import warnings
        with warnings.catch_warnings():
            warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
            self._g.capture_end()
        self.graphs.append(self._g)
        self._g = None

    def _split_at(self, fn):
        self._close()
        self.collectives.append(fn)
        self._open()

    def begin(self):
        global _split, _active
        if _split is not None or _active is not None:
            raise RuntimeError("nested segmented capture")
        self.stream = self._torch.cuda.current_stream()
        self._open()
        _active = self
        if not self.inline:
            _split = self._split_at

    def end(self):
        global _split, _active
        _split = None
        _active = None
        self._close()

    def abort(self):
        """After an exception inside the captured region: leave capture mode."""
        global _split, _active
        _split = None
        _active = None
        if self._g is not None:
            try:
                self._g.capture_end()
            except Exception:
                pass
            self._g = None

    def replay(self):
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.collectives):
                self.collectives[i]()
