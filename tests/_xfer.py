"""The GPU test workers' own host <-> device transfers.

Page-locked by default: the wrong results recorded in rounds 3-4 were 256-byte
holes in the harness's PAGEABLE transfers (torch's pageable copies), not in the
library.  MSX_TEST_PINNED=0 restores pageable transfers; each one then lands
on a prefilled sentinel, so bytes a transfer leaves unwritten read as the
sentinel instead of as whatever the buffer held before."""
import os

import numpy as np
import torch

PINNED = os.environ.get("MSX_TEST_PINNED", "1") != "0"
SENT_DEV, SENT_HOST = 0x5A, 0xA5


def todev(a):
    """numpy array -> a fresh uint8 device tensor holding its bytes."""
    t = torch.empty(max(a.nbytes, 1), dtype=torch.uint8, device="cuda")
    if a.nbytes:
        h = torch.from_numpy(np.frombuffer(a.tobytes(), np.uint8).copy())
        if not PINNED:
            t.fill_(SENT_DEV)
        t.copy_(h.pin_memory() if PINNED else h)
    torch.cuda.synchronize()      # the library's streams do not order after torch's
    return t


def fromdev(t, like, n=None):
    """The first n elements (default like.size) of device tensor t, as a numpy
    array of like's dtype."""
    n = like.size if n is None else n
    h = torch.empty(n * like.dtype.itemsize, dtype=torch.uint8)
    if PINNED:
        h = h.pin_memory()
    else:
        h.fill_(SENT_HOST)
    h.copy_(t[: n * like.dtype.itemsize])
    torch.cuda.synchronize()
    return np.frombuffer(bytearray(h.numpy().tobytes()), like.dtype)


def pinned_dev(a):
    """An independent upload (page-locked source, direct DMA) to compare on the GPU."""
    return torch.from_numpy(np.frombuffer(a.tobytes(), np.uint8).copy()).pin_memory().to("cuda")
