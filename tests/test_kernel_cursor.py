"""Host emulation of the segment-cursor walk of the tile kernels (``csrc/hip/kernels.hip``
``seg_find`` / ``seg_load`` / ``advance``), over the segment tables the kernels really see.

Evidence for VERDICT r2 item 7 (the ``k_crc_tiles<MODE_VERIFY>`` attempt that left a kernel
running on its first GPU run, ``profiles/crc_cols_round2.md``): the verify pass walks every
lane's 16-byte words of a tile with a cursor that only moves forward.  If that walk could loop
forever, or index past the table, for the 100 GB hand-off's table (``bench.py``'s synthetic
AdamW state: 8192-hidden transformer blocks, ~1,500 tensors) or for tables with empty
segments (the hand-off's tensors without an allocation), it would explain the hang.  It does
neither: the walk is bounded by the segments it crosses (+1 per word) and stays in range, so
the cause lies outside the cursor (code generation under the 512-thread register budget is
what remains; the verify stays on ``k_stream_crc<MODE_VERIFY>``)."""
import bisect
import random

ROW = 256 * 16  # TPI_ROW_BYTES: 256 lanes x 16 B
ALIGN = 256     # SEG_ALIGN


def seg_find(offs, pos):
    """Largest i with offs[i] <= pos (the kernel's binary search)."""
    lo, hi = 0, len(offs) - 1
    while lo < hi:
        mid = (lo + hi + 1) >> 1
        if offs[mid] <= pos:
            lo = mid
        else:
            hi = mid - 1
    return lo


def next_off(offs, i):
    return offs[i + 1] if i + 1 < len(offs) else (1 << 64) - 1


def walk_tile(offs, nbytes, gbase, tile_len, lane):
    """One lane's words of one tile, as the kernel visits them; returns (steps, loads)."""
    idx = seg_find(offs, gbase + lane * 16)
    nxt = next_off(offs, idx)
    steps = loads = 0
    for row in range((tile_len + ROW - 1) // ROW):
        rel = row * ROW + lane * 16
        if rel >= tile_len:
            continue
        pos = gbase + rel
        while pos >= nxt:  # advance(): seg_load(idx + 1)
            idx += 1
            assert idx < len(offs), "cursor ran past the segment table"
            nxt = next_off(offs, idx)
            steps += 1
        assert offs[idx] <= pos < nxt
        assert idx == bisect.bisect_right(offs, pos) - 1
        loads += 1
    return steps, loads


def bench_plan(total_bytes=100 * 10 ** 9, hidden=8192):
    """Segment offsets/sizes of bench.synthetic_checkpoint (no tensors allocated)."""
    h = hidden
    ffn = int(8 * h / 3 + 255) // 256 * 256
    block = [(3 * h * h), (h * h), (2 * ffn * h), (h * ffn), h, h]
    offs, sizes, used, off = [], [], 0, 0
    while used < total_bytes:
        for numel in block:
            for esz in (2, 4, 4):  # bf16 param, fp32 exp_avg, fp32 exp_avg_sq
                left = total_bytes - used
                if left <= 0:
                    break
                n = min(numel, max(left // esz, 1))
                offs.append(off)
                sizes.append(n * esz)
                used += n * esz
                off = (off + n * esz + ALIGN - 1) // ALIGN * ALIGN
    return offs, sizes, max(off, ALIGN)


def test_cursor_walk_is_bounded_on_the_100g_plan():
    offs, sizes, total = bench_plan()
    tile = 1 << 20
    ntiles = (total + tile - 1) // tile
    # every tile a segment boundary falls into, plus a random sample and both ends
    boundary_tiles = sorted({o // tile for o in offs} | {0, ntiles - 1})
    rng = random.Random(7)
    tiles = boundary_tiles[:400] + rng.sample(range(ntiles), 100) + boundary_tiles[-50:]
    for t in tiles:
        gbase = t * tile
        tile_len = min(tile, total - gbase)
        crossed = bisect.bisect_right(offs, gbase + tile_len) - bisect.bisect_right(offs, gbase)
        for lane in (0, 1, 17, 128, 255):
            steps, loads = walk_tile(offs, sizes, gbase, tile_len, lane)
            assert steps <= crossed + 1
            assert loads == (tile_len - lane * 16 + ROW - 1) // ROW


def test_cursor_walk_with_empty_and_tiny_segments():
    """Zero-length segments share their offset with the next one (the hand-off's entries
    without an allocation); tiny segments put several inside one 16-byte word's row."""
    rng = random.Random(3)
    offs, off = [], 0
    for _ in range(3000):
        n = rng.choice([0, 0, 1, 16, 255, 256, 4096, 70000])
        offs.append(off)
        off = (off + n + ALIGN - 1) // ALIGN * ALIGN
    total = max(off, ALIGN)
    tile = 1 << 16
    for t in range((total + tile - 1) // tile):
        gbase = t * tile
        tile_len = min(tile, total - gbase)
        for lane in (0, 5, 255):
            steps, _ = walk_tile(offs, None, gbase, tile_len, lane)
            assert steps <= len(offs)
