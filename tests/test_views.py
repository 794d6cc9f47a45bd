"""Non-contiguous tensor views: canonicalisation/classification (csrc/hip/tpi_hip.h kinds)
and host round trips of every kind (the device paths are checked in test_gpu_kernels)."""
import torch

from terraform_provider_iterative_amd.checkpoint import Checkpointer
from terraform_provider_iterative_amd.ops import packing as P
from test_gpu_kernels import _views


def test_canonical_view_merges_and_drops():
    assert P.canonical_view((4, 1, 6), (6, 99, 1)) == [(24, 1)]
    t = torch.zeros(4, 16, 9, 9).contiguous(memory_format=torch.channels_last)
    assert P.canonical_view(t.shape, t.stride()) == [(4, 1296), (16, 1), (81, 16)]
    assert P.canonical_view((1, 1), (5, 7)) == [(1, 1)]


def test_view_classification():
    plan = P.PackPlan.from_tensors(_views("cpu"), tile_bytes=4096)
    kinds = {e.name: int(plan.segs[i]["kind"]) for i, e in enumerate(plan.entries)}
    assert kinds == {"t_f32": P.SEG_TRANSPOSE, "t_bf16": P.SEG_TRANSPOSE, "t_u8": P.SEG_TRANSPOSE,
                     "t_f64": P.SEG_TRANSPOSE, "batched": P.SEG_TRANSPOSE,
                     "channels_last": P.SEG_TRANSPOSE, "rows": P.SEG_ROWS,
                     "rows_aligned": P.SEG_ROWS, "stride2": P.SEG_STRIDED,
                     "expanded": P.SEG_STRIDED, "contig": P.SEG_CONTIG}


def test_all_view_kinds_round_trip_on_host():
    src = _views("cpu")
    ref = {k: v.clone() for k, v in src.items()}
    stream, crcs = P.pack(P.PackPlan.from_tensors(ref, tile_bytes=4096))
    contiguous, _ = P.pack(P.PackPlan.from_tensors(
        {k: v.contiguous() for k, v in ref.items()}, tile_bytes=4096))
    assert (stream == contiguous).all()  # the stream holds the logical (row-major) order
    with Checkpointer(src, tile_bytes=4096, codec="tpz1") as ck:
        ck.save()
        for v in src.values():
            v.zero_()
        assert ck.restore().bad_tiles == 0
    for k in ref:
        assert torch.equal(src[k], ref[k]), k
