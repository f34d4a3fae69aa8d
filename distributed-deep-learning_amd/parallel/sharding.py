"""Parameter-server shard planners.

Reference policies (tensor-granular, each PS owns whole tensors + their Adam slots):

* ``contiguous`` — PS ``r`` owns tensor positions ``[avg*r, avg*(r+1))`` with
  ``avg = T // P``; the last PS also takes the remainder.
  PS side: ``mnist_sync_sharding/parameter_server.py:26-60``;
  worker routing: ``mnist_sync_sharding/worker.py:19-20,30-38,89-94``.
* ``greedy`` — tensors re-ordered by the zig-zag "small, large, 2nd small, 2nd large,
  ..." numel order, then split contiguously.
  ``mnist_sync_sharding_greedy/worker.py:13-37``.
* ``none`` — a single PS owns everything (``mnist_sync/``, ``mnist_async/``).

MI355X-first additions (SURVEY.md §2.8 takeaways):

* ``lpt``  — longest-processing-time bin packing by bytes (tensor-granular).
* ``flat`` — byte-equal split of the flat buffer ignoring tensor boundaries
  (ZeRO-style); with ``P == world`` it maps onto one RCCL reduce-scatter +
  all-gather, the xGMI-optimal pattern.

A plan defines a *plan-ordered* flat buffer: tensors laid out in ``order`` so that every
PS's shard is one contiguous element range ``ps_ranges[p]``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..models.layout import TENSORS, NUM_TENSORS

POLICIES = ("none", "contiguous", "greedy", "lpt", "flat")
FLAT_ALIGN = 64  # elements (256 B): keeps every shard 16-B aligned for dwordx4 access
TENSOR_ALIGN = 64  # elements: every tensor's offset in a plan buffer


def greedy_order(numels: Sequence[int]) -> List[int]:
    """Zig-zag order of ``mnist_sync_sharding_greedy/worker.py:15-30``.

    Indices sorted by numel ascending (stable), then emitted smallest, largest,
    2nd smallest, 2nd largest, ... plus the middle one when the count is odd.
    """
    srt = sorted(range(len(numels)), key=lambda i: numels[i])
    out: List[int] = []
    i, j = 0, len(srt) - 1
    while i < j:
        out.append(srt[i])
        out.append(srt[j])
        i += 1
        j -= 1
    if len(srt) % 2:
        out.append(srt[i])
    return out


def contiguous_counts(total: int, num_ps: int) -> List[int]:
    """Tensors per PS under the reference contiguous split."""
    if num_ps < 1:
        raise ValueError("num_ps must be >= 1")
    if num_ps > total:
        # Reference divides by zero here: reject up front.
        raise ValueError(f"tensor-granular sharding needs num_ps <= {total} tensors, got {num_ps}")
    avg = total // num_ps
    return [avg] * (num_ps - 1) + [avg + total % num_ps]


def reference_route(i: int, total: int, num_ps: int) -> Tuple[int, int]:
    """(owner PS, MPI tag) of the i-th tensor as the reference worker computes it
    (``mnist_sync_sharding/worker.py:30-37``)."""
    avg = total // num_ps
    local_last = avg + total % num_ps
    ind = i // avg
    if i >= total - local_last:
        ind = num_ps - 1
    return ind, i - ind * avg


@dataclass
class ShardPlan:
    policy: str
    num_ps: int
    order: List[int]                       # canonical tensor ids in plan-buffer order
    tensor_offsets: List[int]              # element offset of tensor i (canonical id) in the plan buffer
    ps_ranges: List[Tuple[int, int]]       # [lo, hi) element range owned by each PS
    total: int                             # plan-buffer length in elements (>= model numel)
    owner: Optional[List[int]] = None      # tensor -> PS (tensor-granular policies only)
    meta: Dict[str, object] = field(default_factory=dict)
    # flat policy: bucket ranges of the padded buffer; PS p owns chunk p of every bucket
    bucket_ranges: Optional[List[Tuple[int, int]]] = None

    def ps_segments(self, p: int) -> List[Tuple[int, int]]:
        """All element ranges owned by PS ``p`` (one range for tensor-granular plans)."""
        if self.bucket_ranges is None:
            return [self.ps_ranges[p]]
        segs = []
        for lo, hi in self.bucket_ranges:
            c = (hi - lo) // self.num_ps
            segs.append((lo + p * c, lo + (p + 1) * c))
        return segs

    # ---- queries -------------------------------------------------------------------
    @property
    def tensor_granular(self) -> bool:
        return self.owner is not None

    def shard_numel(self, p: int) -> int:
        return sum(hi - lo for lo, hi in self.ps_segments(p))

    def shard_bytes(self) -> List[int]:
        """Payload bytes per PS (alignment padding excluded for tensor-granular plans)."""
        if self.owner is not None:
            out = [0] * self.num_ps
            for t in TENSORS:
                out[self.owner[t.index]] += t.nbytes
            return out
        return [4 * self.shard_numel(p) for p in range(self.num_ps)]

    def tensor_extent(self, i: int) -> Tuple[int, int]:
        """[lo, hi) of tensor i in the plan buffer including its alignment padding."""
        o = self.tensor_offsets[i]
        return o, o + padded(TENSORS[i].numel)

    def imbalance(self) -> float:
        """max/mean shard bytes (1.0 = perfectly balanced), SURVEY.md §2.8."""
        b = self.shard_bytes()
        return max(b) / (sum(b) / len(b))

    def equal_shards(self) -> bool:
        return len({self.shard_numel(p) for p in range(self.num_ps)}) == 1

    def host_rank(self, p: int, world: int) -> int:
        """Process (= GPU) that hosts PS ``p``.  PS roles are co-located with workers:
        RCCL cannot put two ranks of one communicator on one GPU."""
        return p % world

    def tensors_of(self, p: int) -> List[int]:
        """Tensors owned by PS p (tensor-granular plans only)."""
        if self.owner is None:
            raise ValueError("flat plans split tensors; ownership is by element range")
        return [i for i in self.order if self.owner[i] == p]

    def describe(self) -> str:
        mib = [b / 2**20 for b in self.shard_bytes()]
        return (f"{self.policy} P={self.num_ps} shards(MiB)=" +
                ",".join(f"{m:.2f}" for m in mib) + f" max/mean={self.imbalance():.2f}")


def padded(numel: int) -> int:
    """Tensor extent in the plan buffer: every tensor starts TENSOR_ALIGN-aligned (256 B), so
    the GEMM operand loads and the Adam kernel's 16-B vector path see aligned views, and the
    extents of consecutive tensors stay adjacent (one collective per run of tensors)."""
    return -(-numel // TENSOR_ALIGN) * TENSOR_ALIGN


def _tensor_granular(policy: str, order: List[int], owner: List[int], num_ps: int) -> ShardPlan:
    # owner must be non-decreasing along `order` so each PS's tensors are contiguous.
    numel = [t.numel for t in TENSORS]
    offsets = [0] * NUM_TENSORS
    ranges: List[Tuple[int, int]] = []
    seq: List[int] = []
    pos = 0
    for p in range(num_ps):
        lo = pos
        for i in order:
            if owner[i] == p:
                offsets[i] = pos
                pos += padded(numel[i])
                seq.append(i)
        ranges.append((lo, pos))
    return ShardPlan(policy, num_ps, seq, offsets, ranges, pos, owner=list(owner))


def segment_ps_counts(sizes: Sequence[int], num_ps: int) -> List[int]:
    """PS per group for a segment-aligned flat plan: at least one each, the rest by largest
    remainder of the byte-proportional quota."""
    g = len(sizes)
    if num_ps < g:
        raise ValueError(f"segment-aligned flat plan needs num_ps >= {g} groups, got {num_ps}")
    tot = float(sum(sizes))
    quota = [num_ps * s / tot for s in sizes]
    k = [max(1, int(q)) for q in quota]
    while sum(k) > num_ps:  # the minimum of one pushed the sum over: take from the largest
        i = max((j for j in range(g) if k[j] > 1), key=lambda j: (k[j] - quota[j], k[j]))
        k[i] -= 1
    while sum(k) < num_ps:
        i = max(range(g), key=lambda j: (quota[j] - k[j], sizes[j]))
        k[i] += 1
    return k


def _segment_aligned_flat(num_ps: int, groups: Sequence[Sequence[int]]) -> ShardPlan:
    """Flat plan whose every PS range lies inside ONE group of consecutive tensors (the
    engine's backward segments): an asynchronous worker pushes a PS's shard as soon as its
    segment's gradient exists, so no shard waits for the last segment unless it belongs to it.
    Each group gets ``segment_ps_counts`` PS and is split into that many equal chunks."""
    numel = [t.numel for t in TENSORS]
    gs = [sorted(b) for b in sorted(groups, key=min)]
    if sorted(i for b in gs for i in b) != list(range(NUM_TENSORS)):
        raise ValueError("groups must partition the tensor ids")
    sizes = [sum(padded(numel[i]) for i in b) for b in gs]
    counts = segment_ps_counts(sizes, num_ps)
    offsets = [0] * NUM_TENSORS
    ranges: List[Tuple[int, int]] = []
    pos = 0
    for b, k in zip(gs, counts):
        lo = pos
        for i in b:
            offsets[i] = pos
            pos += padded(numel[i])
        unit = k * FLAT_ALIGN
        pos = lo + -(-(pos - lo) // unit) * unit
        c = (pos - lo) // k
        ranges += [(lo + j * c, lo + (j + 1) * c) for j in range(k)]
    plan = ShardPlan("flat", num_ps, list(range(NUM_TENSORS)), offsets, ranges, pos)
    plan.meta["segment_aligned"] = [len(b) for b in gs]
    plan.meta["ps_per_group"] = counts
    return plan


def host_imbalance(plan: ShardPlan, world: int) -> float:
    """max/mean elements per host process (PS p lives on rank p % world)."""
    load = [0] * world
    for p in range(plan.num_ps):
        load[plan.host_rank(p, world)] += plan.shard_numel(p)
    return max(load) / (sum(load) / world)


def async_groups(segments: Sequence[Sequence[int]], min_frac: float = 0.01) -> List[List[int]]:
    """The backward segments (completion order) as the async plan's PS groups: a segment with
    less than ``min_frac`` of the parameters joins the segment completed after it — it is
    pushed one segment later (harmless: it is tiny) instead of taking a PS of its own, which
    would cost every host a PS at W = 4-8 for a few KB (HIP engine: fc3's 5,130 parameters
    complete alone in segment 0 since fc1 / fc2's weight gradients moved to segment 1)."""
    numel = [t.numel for t in TENSORS]
    total = sum(numel)
    out: List[List[int]] = []
    carry: List[int] = []
    for seg in segments:
        g = carry + list(seg)
        if sum(numel[i] for i in g) < min_frac * total and seg is not segments[-1]:
            carry = g
            continue
        out.append(sorted(g))
        carry = []
    return out


def segment_aligned_num_ps(world: int, groups: Sequence[Sequence[int]],
                           max_imbalance: float = 1.25) -> int:
    """PS count of the async segment-aligned flat plan: the smallest multiple of ``world``
    (every host serves the same number of PS) with a PS per group and per-host load within
    ``max_imbalance`` (else the best of the first four multiples).  W=1: 4, W=2: 6, W=4: 8,
    W=8: 8 with the HIP engine's four segments."""
    best = None
    for m in range(1, 5):
        P = m * world
        if P < len(groups):
            continue
        if P > 64:
            break
        imb = host_imbalance(_segment_aligned_flat(P, groups), world)
        if imb <= max_imbalance:
            return P
        if best is None or imb < best[0]:
            best = (imb, P)
    if best is None:
        raise ValueError(f"no PS count for {len(groups)} groups on {world} ranks")
    return best[1]


def make_plan(policy: str, num_ps: int,
              buckets: Optional[Sequence[Sequence[int]]] = None,
              segment_aligned: bool = False) -> ShardPlan:
    """Build a plan.  ``buckets`` (flat policy only): groups of consecutive canonical
    tensor ids, each padded and split equally over the PSes, so that each bucket can be
    reduce-scattered on its own as soon as backward has produced it.  With
    ``segment_aligned`` the groups are split over DIFFERENT PSes instead (one range per PS,
    the asynchronous PS's layout, ``_segment_aligned_flat``)."""
    policy = policy.lower()
    if policy not in POLICIES:
        raise ValueError(f"unknown shard policy {policy!r}; choose from {POLICIES}")
    if segment_aligned:
        if policy != "flat" or buckets is None:
            raise ValueError("segment_aligned applies to the flat policy with buckets")
        return _segment_aligned_flat(num_ps, buckets)
    numel = [t.numel for t in TENSORS]
    if policy == "none":
        if num_ps != 1:
            # mnist_sync/worker.py:49 hard-codes one PS.
            raise ValueError("shard policy 'none' means exactly one parameter server")
        return _tensor_granular("none", list(range(NUM_TENSORS)), [0] * NUM_TENSORS, 1)
    if policy in ("contiguous", "greedy"):
        order = list(range(NUM_TENSORS)) if policy == "contiguous" else greedy_order(numel)
        counts = contiguous_counts(NUM_TENSORS, num_ps)
        owner = [0] * NUM_TENSORS
        pos = 0
        for p, c in enumerate(counts):
            for i in order[pos:pos + c]:
                owner[i] = p
            pos += c
        plan = _tensor_granular(policy, order, owner, num_ps)
        plan.meta["reference_order"] = order
        return plan
    if policy == "lpt":
        if num_ps > NUM_TENSORS:
            raise ValueError(f"lpt needs num_ps <= {NUM_TENSORS}")
        load = [0] * num_ps
        owner = [0] * NUM_TENSORS
        for i in sorted(range(NUM_TENSORS), key=lambda i: (-numel[i], i)):
            p = min(range(num_ps), key=lambda q: (load[q], q))
            owner[i] = p
            load[p] += numel[i]
        return _tensor_granular("lpt", list(range(NUM_TENSORS)), owner, num_ps)
    # flat: canonical order, every bucket padded to a multiple of P*FLAT_ALIGN and split
    # into P equal chunks.
    if buckets is None:
        buckets = [list(range(NUM_TENSORS))]
    flat_ids = [i for b in buckets for i in b]
    if sorted(flat_ids) != list(range(NUM_TENSORS)):
        raise ValueError("buckets must partition the tensor ids")
    unit = num_ps * FLAT_ALIGN
    offsets = [0] * NUM_TENSORS
    branges: List[Tuple[int, int]] = []
    pos = 0
    for b in sorted(buckets, key=min):
        lo = pos
        for i in sorted(b):
            offsets[i] = pos
            pos += padded(numel[i])
        pos = lo + -(-(pos - lo) // unit) * unit
        branges.append((lo, pos))
    plan = ShardPlan("flat", num_ps, list(range(NUM_TENSORS)), offsets, [], pos,
                     bucket_ranges=branges)
    plan.ps_ranges = [plan.ps_segments(p)[0] for p in range(num_ps)] if len(branges) == 1 else []
    plan.meta["buckets"] = [sorted(b) for b in sorted(buckets, key=min)]
    return plan


def balance_table(max_ps: int = 8) -> List[Dict[str, object]]:
    """Replays SURVEY.md §2.8 for every policy and P in 1..max_ps."""
    rows = []
    for p in range(1, max_ps + 1):
        row: Dict[str, object] = {"P": p}
        for pol in ("contiguous", "greedy", "lpt", "flat"):
            plan = make_plan(pol, p)
            row[pol] = round(plan.imbalance(), 2)
        rows.append(row)
    return rows
