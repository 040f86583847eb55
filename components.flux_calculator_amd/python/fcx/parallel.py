"""Multi-GPU layout of the flux path: contiguous cell ranges per rank and the
exchange -> atmosphere accumulation completed by ONE all-reduce.

Partition rules of the reference:
  * apple_range: decomp_def.F90:23-31 (APPLE): rank r < P-1 owns [r*floor(N/P), +floor(N/P)),
    the last rank the remainder; the offset/size pair is what flux_calculator declares to
    OASIS as the APPLE partition [1, offset, size] (flux_calculator.F90:801-803).
  * task_range: read_scrip_grid_dimensions (flux_calculator_io.F90:77-107): the cells whose
    `task` entry equals the rank; offset = first such cell - 1, an empty task gets (0, 0).

Exchange -> atmosphere accumulation: every exchange cell lies in exactly one atmosphere cell
(the exchange grid is the intersection of the atmosphere and bottom grids), with weight
area_x / area_a, and the exchange grid is ordered by atmosphere row, so the cells of one
atmosphere cell are contiguous.  A rank's contiguous exchange range therefore touches a
contiguous atmosphere range whose first and last cells may be shared with the neighbour
ranks -- the only cross-rank exchange of the whole path.  Each rank writes its partial sums
of those two cells into boundary slots of a [P-1][stride] buffer (zero elsewhere); one
all-reduce (sum) over the ranks completes them.
"""
from dataclasses import dataclass

import numpy as np


def apple_range(n_global, rank, nranks):
    """(offset, size) of rank's cells, decomp_def.F90:23-31 with id_jm = 1 row per cell."""
    if not 0 <= rank < nranks:
        raise ValueError(f"rank {rank} outside 0..{nranks - 1}")
    part = n_global // nranks
    offset = rank * part
    size = part if rank < nranks - 1 else n_global - rank * part
    return offset, size


def task_range(task, mype):
    """(offset, size) from the exchange-grid `task` vector (flux_calculator_io.F90:77-107)."""
    task = np.asarray(task)
    hit = np.nonzero(task == mype)[0]
    if hit.size == 0:
        return 0, 0
    return int(hit[0]), int(hit.size)


def task_ranges(task, nranks):
    """Every rank's (offset, size, right_slot) from the `task` vector (io:77-107).

    A rank may own no cells (io:101-104).  The boundary slot between two ranks is numbered
    by the rank on its right minus one, so a rank's right slot is that of the next rank WITH
    cells: an empty rank between two shards that share an atmosphere cell must not split
    their partial sums into two slots."""
    r = [task_range(task, m) for m in range(nranks)]
    out = []
    for m, (off, size) in enumerate(r):
        nxt = next((k for k in range(m + 1, nranks) if r[k][1] > 0), None)
        out.append((off, size, (nxt - 1) if nxt is not None else m))
    return out


@dataclass
class AtmosMap:
    """Global exchange -> atmosphere map: atmos_index[x] non-decreasing, weight[x]."""
    atmos_index: np.ndarray  # int32 [n_exchange]
    weight: np.ndarray  # float64 [n_exchange]
    n_atmos: int


def synthetic_atmos_map(n_exchange, cells_per_atmos=4, seed=20231015):
    """1 atmosphere cell per ~4 exchange cells: run lengths 3..5,
    exchange cells ordered by atmosphere cell, weights = exchange area / atmosphere area."""
    rng = np.random.Generator(np.random.PCG64([seed, 99]))
    lengths = rng.integers(cells_per_atmos - 1, cells_per_atmos + 2, n_exchange // max(cells_per_atmos - 1, 1) + 2)
    while lengths.sum() < n_exchange:  # (only with runs that may be empty: cells_per_atmos 1)
        lengths = np.concatenate([lengths, rng.integers(cells_per_atmos - 1, cells_per_atmos + 2, n_exchange + 2)])
    ends = np.cumsum(lengths)
    n_atmos = int(np.searchsorted(ends, n_exchange, side="left")) + 1
    idx = np.repeat(np.arange(n_atmos, dtype=np.int32), lengths[:n_atmos])[:n_exchange]
    area = rng.uniform(0.5, 1.5, n_exchange)
    tot = np.bincount(idx, weights=area, minlength=n_atmos)
    w = area / tot[idx]
    return AtmosMap(np.ascontiguousarray(idx, dtype=np.int32), np.ascontiguousarray(w), n_atmos)


@dataclass
class LocalAtmos:
    """A rank's view: local atmosphere indices of its exchange range and its boundary slots."""
    offset: int  # first exchange cell (0-based global)
    size: int
    atmos_offset: int  # first local atmosphere cell (global index)
    n_atmos: int
    atmos_index: np.ndarray  # int32 [size], 0-based local
    weight: np.ndarray
    left: int  # boundary slot of the first local atmosphere cell, -1 = not shared
    right: int  # boundary slot of the last one, -1 = not shared
    n_boundaries: int


def boundary_slots(ranges, index_at):
    """Every rank's (left, right) boundary slots for contiguous exchange ranges in rank order.

    ranges: every rank's (offset, size); index_at(x): global atmosphere cell of exchange cell
    x.  Boundary m - 1 is the one just before rank m's cells (an empty rank has no boundary
    of its own: the next rank with cells numbers it).  All ranks that hold part of one
    atmosphere cell use ONE slot, that of the first rank boundary inside the cell, so a rank
    whose cells all lie in an atmosphere cell shared with both neighbours gets left == right
    and the one all-reduce sums the cell over three or more ranks."""
    left, right = [-1] * len(ranges), [-1] * len(ranges)
    prev, a0s, a1s = None, {}, {}
    for k, (off, size) in enumerate(ranges):
        if size == 0:
            continue
        a0, a1 = int(index_at(off)), int(index_at(off + size - 1))
        if prev is not None and a1s[prev] == a0:  # the boundary before rank k cuts a cell
            chained = left[prev] >= 0 and a0s[prev] == a1s[prev]  # the cell began before prev
            slot = left[prev] if chained else k - 1
            right[prev] = left[k] = slot
        a0s[k], a1s[k] = a0, a1
        prev = k
    return list(zip(left, right))


def local_atmos(amap: AtmosMap, rank, nranks, offset=None, size=None, right_slot=None, ranges=None):
    """right_slot: the slot of the boundary after this rank's cells (default `rank`; with
    empty ranks in between, task_ranges gives it).  ranges: every rank's (offset, size); with
    them (or with APPLE ranges, offset None) the slots come from boundary_slots, which also
    serves a rank inside one atmosphere cell shared with both neighbours."""
    n_global = amap.atmos_index.shape[0]
    if ranges is None and offset is None:
        ranges = [apple_range(n_global, r, nranks) for r in range(nranks)]
    if ranges is not None:
        offset, size = ranges[rank]
    gi = amap.atmos_index[offset: offset + size]
    if size == 0:
        return LocalAtmos(offset, 0, 0, 0, np.zeros(0, np.int32), np.zeros(0), -1, -1, max(nranks - 1, 0))
    a0, a1 = int(gi[0]), int(gi[-1])
    if ranges is not None:
        left, right = boundary_slots(ranges, lambda x: amap.atmos_index[x])[rank]
    else:
        left = rank - 1 if (offset > 0 and amap.atmos_index[offset - 1] == a0) else -1
        end = offset + size
        right_slot = rank if right_slot is None else right_slot
        right = right_slot if (end < n_global and amap.atmos_index[end] == a1) else -1
        if left >= 0 and right >= 0 and a0 == a1:
            raise ValueError(f"rank {rank}: its {size} cells lie inside one atmosphere cell shared "
                             "with both neighbours: pass every rank's ranges to give it one slot")
    return LocalAtmos(offset, size, a0, a1 - a0 + 1, np.ascontiguousarray(gi - a0, dtype=np.int32),
                      np.ascontiguousarray(amap.weight[offset: offset + size]), left, right,
                      max(nranks - 1, 0))


def pack_boundaries(la: LocalAtmos, partial_fields, stride):
    """CPU form of the engine's boundary write: [n_boundaries][stride] with this rank's partial
    sums of its shared first/last atmosphere cells (fields in columns), zero elsewhere."""
    buf = np.zeros((la.n_boundaries, stride))
    for f, out in enumerate(partial_fields):
        if la.left >= 0:
            buf[la.left, f] = out[0]
        if la.right >= 0:
            buf[la.right, f] = out[-1]
    return buf


def unpack_boundaries(la: LocalAtmos, reduced, fields):
    """CPU form of fcx_atmos_finish: completed boundary sums back into the local fields."""
    for f, out in enumerate(fields):
        if la.left >= 0:
            out[0] = reduced[la.left, f]
        if la.right >= 0:
            out[-1] = reduced[la.right, f]
    return fields


class PeriodicAtmosMap:
    """Structured synthetic map for large sharded runs: every 16 exchange cells form 4
    atmosphere cells of 3, 4, 5 and 4 cells (mean 4).  Any rank builds
    its own range in O(size) without the global arrays; areas come from an integer hash of
    the global cell index, weights = area / sum of the atmosphere cell's areas."""
    LENGTHS = (3, 4, 5, 4)
    PERIOD = 16

    def __init__(self):
        starts = np.cumsum((0,) + self.LENGTHS[:-1])
        self._sub = np.repeat(np.arange(4), self.LENGTHS)  # cell in period -> sub-cell
        self._start = starts[self._sub]  # first cell of the sub-cell inside the period
        self._len = np.array(self.LENGTHS)[self._sub]

    def index(self, x):
        x = np.asarray(x, dtype=np.int64)
        return (x // self.PERIOD) * 4 + self._sub[x % self.PERIOD]

    @staticmethod
    def area(x):
        h = (np.asarray(x, dtype=np.uint64) * np.uint64(2654435761)) % np.uint64(1000003)
        return 0.5 + h.astype(np.float64) / 1000003.0

    def weight(self, x, n_global):
        x = np.asarray(x, dtype=np.int64)
        first = (x // self.PERIOD) * self.PERIOD + self._start[x % self.PERIOD]
        length = self._len[x % self.PERIOD]
        tot = np.zeros(x.shape)
        for k in range(5):
            y = first + k
            tot += np.where((k < length) & (y < n_global), self.area(y), 0.0)
        return self.area(x) / tot

    def local(self, offset, size, rank, nranks, n_global, right_slot=None, ranges=None):
        """right_slot: the boundary slot after this rank's cells (default `rank`; with empty
        ranks in the decomposition, the next rank with cells minus one, as task_ranges).
        ranges: every rank's (offset, size): slots from boundary_slots."""
        right_slot = rank if right_slot is None else right_slot
        x = np.arange(offset, offset + size, dtype=np.int64)
        gi = self.index(x)
        if size == 0:
            return LocalAtmos(offset, 0, 0, 0, np.zeros(0, np.int32), np.zeros(0), -1, -1, max(nranks - 1, 0))
        a0, a1 = int(gi[0]), int(gi[-1])
        if ranges is not None:
            left, right = boundary_slots(ranges, lambda c: int(self.index(c)))[rank]
        else:
            left = rank - 1 if (offset > 0 and int(self.index(offset - 1)) == a0) else -1
            end = offset + size
            right = right_slot if (end < n_global and int(self.index(end)) == a1) else -1
        return LocalAtmos(offset, size, a0, a1 - a0 + 1, np.ascontiguousarray(gi - a0, dtype=np.int32),
                          np.ascontiguousarray(self.weight(x, n_global)), left, right, max(nranks - 1, 0))

    def global_map(self, n_global):
        x = np.arange(n_global, dtype=np.int64)
        idx = self.index(x)
        return AtmosMap(np.ascontiguousarray(idx, dtype=np.int32), self.weight(x, n_global),
                        int(idx[-1]) + 1 if n_global else 0)


class BlockedRandomAtmosMap:
    """Runs of 3, 4 or 5 exchange cells per atmosphere cell in random order, so that the
    segments cross the fused kernel's 128-cell wave tiles at random places, as on an
    intersection grid: every block of 4096 exchange cells holds 1024 atmosphere cells (341
    runs of 3, 342 of 4 and 341 of 5, shuffled by a generator seeded with the block index).
    Any rank builds its own range in O(size) without the global arrays (a global random-run
    map is O(n_global) per rank: 80M cells at 8 x 10M).  Areas as PeriodicAtmosMap, weights =
    area / sum of the atmosphere cell's areas (the last block truncated at n_global)."""
    BLOCK = 4096
    RUNS = 1024
    COUNTS = (341, 342, 341)  # runs of 3, 4, 5 cells: 1024 runs, 4096 cells

    def __init__(self, seed=20231015):
        self.seed = seed
        self._base = np.repeat(np.array([3, 4, 5]), self.COUNTS)

    def _runs(self, b):
        lengths = self._base.copy()
        np.random.default_rng([self.seed, 11, int(b)]).shuffle(lengths)
        return np.repeat(np.arange(self.RUNS, dtype=np.int64), lengths)  # run of every cell of the block

    def _cells(self, lo, hi, n_global):
        """global atmosphere index and weight of cells [lo, hi)"""
        if hi <= lo:
            return np.zeros(0, np.int64), np.zeros(0)
        b0, b1 = lo // self.BLOCK, (hi - 1) // self.BLOCK
        idx = np.concatenate([self._runs(b) + b * self.RUNS for b in range(b0, b1 + 1)])
        x = np.arange(b0 * self.BLOCK, min((b1 + 1) * self.BLOCK, n_global), dtype=np.int64)
        idx = idx[: x.size]
        area = PeriodicAtmosMap.area(x)
        first = idx[0]
        tot = np.bincount(idx - first, weights=area)
        w = area / tot[idx - first]
        s = lo - b0 * self.BLOCK
        return idx[s: s + (hi - lo)], w[s: s + (hi - lo)]

    def local(self, offset, size, rank, nranks, n_global, right_slot=None, ranges=None):
        """right_slot, ranges: as PeriodicAtmosMap.local."""
        right_slot = rank if right_slot is None else right_slot
        if size == 0:
            return LocalAtmos(offset, 0, 0, 0, np.zeros(0, np.int32), np.zeros(0), -1, -1, max(nranks - 1, 0))
        lo, hi = max(offset - 1, 0), min(offset + size + 1, n_global)  # one neighbour cell each side
        gi, w = self._cells(lo, hi, n_global)
        mine = slice(offset - lo, offset - lo + size)
        g, wm = gi[mine], w[mine]
        a0, a1 = int(g[0]), int(g[-1])
        if ranges is not None:
            left, right = boundary_slots(ranges, lambda c: int(self._cells(c, c + 1, n_global)[0][0]))[rank]
        else:
            left = rank - 1 if (offset > 0 and int(gi[0]) == a0) else -1
            right = right_slot if (offset + size < n_global and int(gi[-1]) == a1) else -1
        return LocalAtmos(offset, size, a0, a1 - a0 + 1, np.ascontiguousarray(g - a0, dtype=np.int32),
                          np.ascontiguousarray(wm), left, right, max(nranks - 1, 0))

    def global_map(self, n_global):
        idx, w = self._cells(0, n_global, n_global)
        return AtmosMap(np.ascontiguousarray(idx, dtype=np.int32), np.ascontiguousarray(w),
                        int(idx[-1]) + 1 if n_global else 0)


@dataclass
class ModelMap:
    """Exchange -> model (e.g. ocean) remap links, SCRIP style: 0-based src (exchange cell),
    dst (model cell) and weight, in file order."""
    src: np.ndarray
    dst: np.ndarray
    weight: np.ndarray
    n_model: int


def synthetic_model_map(n_exchange, n_model, links_per_cell=1, seed=20231016):
    """Every exchange cell lies in one model cell (conservative weights area_x / area_model).
    The exchange grid follows the atmosphere rows, so a model cell is met in several short
    runs scattered along it: runs of 1..8 exchange cells, each in a random model cell.
    links_per_cell=2 adds a second, distance-weighted link per exchange cell (the two weights
    summing to the conservative one), as a non-conservative remap has; links in a shuffled
    file order."""
    if links_per_cell not in (1, 2):
        raise ValueError(f"links_per_cell must be 1 or 2, got {links_per_cell}")
    if n_model < links_per_cell:
        raise ValueError(f"{links_per_cell} links per exchange cell need as many model cells, got {n_model}")
    rng = np.random.Generator(np.random.PCG64([seed, 7]))
    lengths = rng.integers(1, 9, n_exchange // 4 + 2)
    while lengths.sum() < n_exchange:  # (short draws on small grids: more runs until they cover it)
        lengths = np.concatenate([lengths, rng.integers(1, 9, n_exchange // 4 + 2)])
    lengths = lengths[: int(np.searchsorted(np.cumsum(lengths), n_exchange)) + 1]
    owner = np.repeat(rng.integers(0, n_model, lengths.size), lengths)[:n_exchange]
    area = rng.uniform(0.5, 1.5, n_exchange)
    tot = np.bincount(owner, weights=area, minlength=n_model)
    w = area / tot[owner]
    src = np.arange(n_exchange, dtype=np.int64)
    if links_per_cell == 1:
        return ModelMap(src.astype(np.int32), owner.astype(np.int32), w, n_model)
    other = (owner + rng.integers(1, n_model, n_exchange)) % n_model
    f = rng.uniform(0.6, 0.9, n_exchange)
    s2 = np.stack([src, src], 1).reshape(-1)
    d2 = np.stack([owner, other], 1).reshape(-1)
    w2 = np.stack([w * f, w * (1 - f)], 1).reshape(-1)
    perm = rng.permutation(s2.size)
    return ModelMap(s2[perm].astype(np.int32), d2[perm].astype(np.int32), w2[perm], n_model)


def local_links(mmap: ModelMap, offset, size):
    """The links whose exchange cell is in this rank's range, src made local (0-based); dst
    stays global: every rank writes partial sums of the whole model grid and one all-reduce
    of the outputs completes them."""
    keep = (mmap.src >= offset) & (mmap.src < offset + size)
    return (np.ascontiguousarray(mmap.src[keep] - offset, dtype=np.int32),
            np.ascontiguousarray(mmap.dst[keep], dtype=np.int32), np.ascontiguousarray(mmap.weight[keep]))


def geometric_maps(n_atmos_side, ocean_ratio=0.75, offset=(0.3, 0.45)):
    """Exchange grid of two overlapping regular grids, as the IOW ESM builds it: the
    intersection of an atmosphere grid (n_atmos_side^2 unit cells) with a finer ocean grid
    (cells of ocean_ratio, shifted by offset), one exchange cell per non-empty (atmosphere,
    ocean) pair, ordered by atmosphere row, atmosphere column, then ocean row and column
    (the exchange grid follows the atmosphere rows).  Returns the exchange ->
    atmosphere map (contiguous runs, weights = area / atmosphere cell area) and the
    conservative exchange -> ocean remap (one link per exchange cell, weights = area /
    ocean cell area, links in exchange order), so a model cell's links come from a few
    atmosphere rows, as on the real grids.  About (1 + 1/ocean_ratio)^2 exchange cells per
    atmosphere cell."""
    na = int(n_atmos_side)

    def axis(off):
        lo = off - ocean_ratio * np.ceil(off / ocean_ratio)  # first ocean edge <= 0
        n_o = int(np.ceil((na - lo) / ocean_ratio))
        edges = np.unique(np.concatenate([np.arange(na + 1, dtype=np.float64), lo + ocean_ratio * np.arange(n_o + 1)]))
        edges = edges[(edges >= 0) & (edges <= na)]
        mid = 0.5 * (edges[:-1] + edges[1:])
        width = np.diff(edges)
        keep = width > 1e-12
        ia = np.floor(mid[keep]).astype(np.int64)
        io = np.floor((mid[keep] - lo) / ocean_ratio).astype(np.int64)
        return ia, io, width[keep], n_o

    ax, ox, wx, nox = axis(offset[0])
    ay, oy, wy, noy = axis(offset[1])
    # every (y-segment, x-segment) pair is one exchange cell
    sy, sx = np.meshgrid(np.arange(ay.size), np.arange(ax.size), indexing="ij")
    sy, sx = sy.ravel(), sx.ravel()
    order = np.lexsort((ox[sx], oy[sy], ax[sx], ay[sy]))  # last key is the primary one
    sy, sx = sy[order], sx[order]
    area = wy[sy] * wx[sx]
    a_idx = (ay[sy] * na + ax[sx]).astype(np.int32)
    o_idx = (oy[sy] * nox + ox[sx]).astype(np.int64)
    n_model = int(noy * nox)
    a_w = area / np.bincount(a_idx, weights=area, minlength=na * na)[a_idx]
    o_w = area / np.bincount(o_idx, weights=area, minlength=n_model)[o_idx]
    n = area.size
    return (AtmosMap(np.ascontiguousarray(a_idx), np.ascontiguousarray(a_w), na * na),
            ModelMap(np.arange(n, dtype=np.int32), o_idx.astype(np.int32), np.ascontiguousarray(o_w), n_model))
