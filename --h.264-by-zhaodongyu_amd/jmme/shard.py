"""Multi-GPU partitioning of the motion-estimation path.

JM's ME for frame t searches the reconstruction of t-1 (store_picture_in_dpb,
JM/lencod/src/mbuffer.c:1905), so frames of one GOP are sequential.  Two ways
to use N GPUs, one process per GPU, torch.distributed over RCCL:

* GOP shard ("gop", weak scaling): closed GOPs (IDRPeriod) are dealt
  round-robin; each rank owns its frames, references and jmme context, and
  nothing crosses ranks on the data path.  `gop_owner`.
* Band shard ("band", strong scaling of one stream): the rank that owns the
  encoder loop (src) broadcasts the current frame and the reconstructed
  reference -- one padded 8-bit plane each, RCCL broadcast over xGMI -- and
  every rank searches the macroblock-row band `band_rows` gives it against the
  whole reference (search windows cross band borders, so each rank needs the
  full plane, not a halo).  The per-partition results are all-gathered back
  in band order, which is raster order.

The thesis's fractal P-frame coder shards the same way, without the
sequential dependency inside a frame: range blocks carry no predictor
(encode_Oneframe, ZL/src/image.c:1108-1127), so each rank takes a band of
macroblock (or 4x4 range-block) rows, the src rank broadcasts the range plane
and the reference (domain) views, every rank builds its own domain images
(words / box sums) from the received planes, searches its band against the
whole reference, and the per-macroblock trees (or per-block results) are
all-gathered in raster order.  `fractal_band_step`.

Nothing here computes a search: the caller passes the engine call, so the
same bookkeeping runs on RCCL with the HIP engine and on gloo in the CPU
tests.
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np
import torch
import torch.distributed as dist


def gop_owner(gop: int, world_size: int) -> int:
    """Rank that encodes closed GOP `gop` (round-robin)."""
    return gop % world_size


def band_rows(mb_rows: int, rank: int, world_size: int) -> tuple[int, int]:
    """[r0, r1) macroblock rows of `rank`'s band: contiguous, sizes differ by at most one."""
    r0 = mb_rows * rank // world_size
    r1 = mb_rows * (rank + 1) // world_size
    return r0, r1


def band_units(mb_y: np.ndarray, rank: int, world_size: int, mb_rows: int) -> np.ndarray:
    """Indices of the units (MB x ref requests, `mb_y` in pels) that `rank` searches."""
    r0, r1 = band_rows(mb_rows, rank, world_size)
    row = np.asarray(mb_y) // 16
    return np.nonzero((row >= r0) & (row < r1))[0]


def _distributed(group=None) -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def broadcast_planes(planes: Sequence[torch.Tensor], src: int = 0, group=None) -> None:
    """In-place broadcast of the src rank's planes (current frame, reconstructed
    reference) to every rank; tensors must have the same shape and dtype everywhere."""
    if not _distributed(group):
        return
    for p in planes:
        dist.broadcast(p, src=src, group=group)


def gather_bands(local: torch.Tensor, counts: Sequence[int], group=None) -> torch.Tensor:
    """All-gather each rank's result rows (`local`: [counts[rank], ...]) into one
    tensor in rank order; ragged bands are padded to the largest for the collective."""
    ws = len(counts)
    if not _distributed(group):
        return local[:counts[0]]
    width = max(counts)
    pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([parts[r][:counts[r]] for r in range(ws)])


def band_exchange(planes: Sequence[torch.Tensor], d_out_band: torch.Tensor, counts: Sequence[int],
                  work: Callable[[], None], src: int = 0, group=None) -> torch.Tensor:
    """Broadcast the planes, run this rank's band (`work()` enqueues it on the
    current stream, writing d_out_band[:counts[rank]]), all-gather every
    band's rows in rank order."""
    broadcast_planes(planes, src=src, group=group)
    work()
    return gather_bands(d_out_band, counts, group=group)


def fractal_band_step(planes: Sequence[torch.Tensor], d_out_band: torch.Tensor, counts: Sequence[int],
                      encode_band: Callable[[torch.Tensor], None], src: int = 0, group=None) -> torch.Tensor:
    """One band-sharded fractal P-frame: broadcast [range plane, view 0, view 1, ...],
    encode this rank's band (`encode_band(d_out_band)` builds the local domain
    images from the received views and encodes the band's rows), all-gather the
    bands' records (raster order)."""
    return band_exchange(planes, d_out_band, counts, lambda: encode_band(d_out_band), src=src, group=group)


def band_step(planes: Sequence[torch.Tensor], d_req_band: torch.Tensor, n_band: int, d_out_band: torch.Tensor,
              counts: Sequence[int], search: Callable[[torch.Tensor, int, torch.Tensor], None],
              src: int = 0, group=None) -> torch.Tensor:
    """One band-sharded frame: broadcast the planes, search this rank's band,
    all-gather every band's results (raster order).  `search(d_req, n, d_out)`
    enqueues the engine call on the current stream."""
    return band_exchange(planes, d_out_band, counts, lambda: search(d_req_band, n_band, d_out_band), src=src,
                         group=group)
