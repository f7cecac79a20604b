"""Multi-GPU search: owned-k sharding and the hit gather.

The reference's only parallelism is a ProcessPoolExecutor over overlapping
chunks of one record (src/merpcr/core/engine.py:386-422), whose results come
back by pickling.  Here one process drives one GPU (torch.distributed, backend
"nccl" = RCCL over xGMI on MI355X, "gloo" on CPU for tests):

* ``shard_ranges`` splits the genome's (sequence, amplicon start k) space into
  contiguous owned ranges of equal base count.  Every rank can hold the whole
  genome (it is tiny next to 288 GB of HBM); each scans only the windows its
  owned k need, and all boundary tests use the true record length, so the
  union of the ranks' hits is exactly the single-GPU hit list.
* Owned ranges are ordered and hit order never crosses a range boundary, so the
  rank-ordered concatenation of per-rank sorted lists is the global order.
  The gatherv of the GPU path lives in the library (``native_comm`` ->
  mp_comm_gather_hits: an RCCL all-gather of the counts, then one grouped
  ncclSend/ncclRecv per rank into rank 0's buffer); ``gather_hits`` is the same
  exchange over torch.distributed, for gloo (CPU tests, ranks sharing one GPU,
  which RCCL does not admit).  There is no other data-path collective.
* Contig sharding (``contig_shards``): each rank holds only its own whole
  records (a contiguous run of the file's records, balanced by bases) and
  scans them completely; ``gather_hits(..., seq_base=first record)`` shifts
  the rank-local record index to the file's before the gatherv, so rank 0
  again receives the file-ordered hit list.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

HIT_BYTES = 24


def shard_ranges(lengths: Sequence[int], world: int) -> List[Tuple[int, int, int, int]]:
    """Owned ranges (seq_begin, seq_end, k_begin, k_end) for each rank."""
    lens = np.asarray(lengths, dtype=np.int64)
    cum = np.concatenate([[0], np.cumsum(lens)])
    total = int(cum[-1])
    n_seq = len(lens)

    def locate(g: int):
        if g >= total:
            return n_seq, 0
        s = int(np.searchsorted(cum, g, side="right") - 1)
        return s, g - int(cum[s])

    out = []
    for r in range(world):
        a = total * r // world
        b = total * (r + 1) // world
        sa, ka = locate(a)
        sb, kb = locate(b)
        out.append((sa, sb, ka, kb))
    return out


def contig_shards(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous record ranges [first, last) per rank, balanced by bases (whole records)."""
    lens = np.asarray(lengths, dtype=np.int64)
    cum = np.concatenate([[0], np.cumsum(lens)])
    total = int(cum[-1])
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, total * r // world, side="left"))
        cuts.append(min(max(c, cuts[-1]), len(lens)))
    cuts.append(len(lens))
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def native_comm(device: int, group=None):
    """This rank's RCCL communicator inside libmerpcr_hip (mp_comm_create), for the
    process-per-GPU layout: rank 0 makes the 128-byte unique id, torch.distributed (any
    backend, e.g. gloo) carries it to the other ranks -- plumbing only; the hit gather
    itself (mp_comm_gather_hits) is a grouped ncclSend/ncclRecv over xGMI."""
    import torch.distributed as dist
    from ._native import Comm, comm_unique_id
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [None]
    if rank == 0:  # an error travels in the broadcast, so no rank is left waiting in it
        try:
            obj = [("ok", comm_unique_id())]
        except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
            obj = [("err", f"rank 0 could not make the RCCL id: {type(e).__name__}: {e}")]
    dist.broadcast_object_list(obj, src=0, group=group)
    kind, payload = obj[0]
    if kind == "err":
        raise RuntimeError(payload)
    return Comm(payload, world, rank, device)


class IpcGather:
    """Hit gather to rank 0 by the copy engines, for one process per GPU on one node.

    Rank 0 allocates ``slots`` x ``world`` fixed regions of ``cap`` hits (the largest any rank
    asks for) and as many count words in its HBM and exports both (mp_ipc_handle);
    torch.distributed (any backend: the control plane) carries the handles; every other rank
    maps them on its own device (mp_ipc_open).  After a completed run, ``put`` copies the run's
    hits into this rank's region of the given slot and its count into the slot's word, on the
    given stream (mp_search_put_hits: no kernel on the CUs, no collective, no host
    synchronisation between ranks).  Pipelined search handles each put into a slot of their
    own, so no two streams of a rank ever write one region.  A run with more hits than ``cap``
    is not copied; ``settle`` (collective, after the ranks' streams are synchronised) then
    regrows every region to twice the largest need and every rank puts each slot's last run
    again.  Rank 0's ``hits(slot)`` is then the rank-ordered concatenation (the contig-shard
    sequence shift applied there, so no rank's own list is modified).  Collective to create
    (every rank), like the RCCL communicator it stands beside; a failure to export or to map
    raises on every rank, after the handles' broadcast."""

    def __init__(self, device: int, cap: int, group=None, slots: int = 1):
        import torch.distributed as dist
        self.device, self.group, self.slots = device, group, max(1, int(slots))
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        caps = [None] * self.world  # one region size for every rank: the largest asked for
        dist.all_gather_object(caps, int(cap), group=group)
        self.cap = max(caps)
        self._opened = []
        self._buf = self._cnt = None
        self._last = {}   # slot -> (search, stream) of this rank's last put there
        self._need = 0    # the largest count a put of this rank could not copy (0: none)
        self.regrowths = 0
        self._map()

    def _map(self):
        """Rank 0 allocates and exports; the others map.  An export failure travels in the
        broadcast itself, so every rank leaves the collective before raising it."""
        import torch
        import torch.distributed as dist
        from . import _native
        if self.rank == 0:
            try:
                dev = torch.device("cuda", self.device)
                n = self.slots * self.world
                self._buf = torch.empty(n * self.cap * HIT_BYTES, dtype=torch.uint8, device=dev)
                self._cnt = torch.zeros(n, dtype=torch.int64, device=dev)
                obj = [("ok", (_native.ipc_handle(self._buf.data_ptr()), _native.ipc_handle(self._cnt.data_ptr())))]
            except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
                obj = [("err", f"rank 0 could not export its gather buffers: {type(e).__name__}: {e}")]
        else:
            obj = [None]
        dist.broadcast_object_list(obj, src=0, group=self.group)
        kind, payload = obj[0]
        if kind == "err":
            raise RuntimeError(payload)
        if self.rank == 0:
            self._base, self._cbase = self._buf.data_ptr(), self._cnt.data_ptr()
        else:  # each handle maps its whole allocation: add the tensor's offset in it
            (hb, ob), (hc, oc) = payload
            mb = _native.ipc_open(hb, self.device)
            self._opened.append(mb)
            mc = _native.ipc_open(hc, self.device)
            self._opened.append(mc)
            self._base, self._cbase = mb + ob, mc + oc

    def _region(self, slot: int):
        i = slot * self.world + self.rank
        return self._base + i * self.cap * HIT_BYTES, self._cbase + i * 8

    def put(self, search, stream=None, slot: int = 0) -> bool:
        """This rank's last run of `search` into its region of `slot`.  False: more hits than
        the region holds (nothing copied; ``settle`` regrows and puts it again)."""
        from . import _native
        self._last[slot] = (search, stream)
        region, count = self._region(slot)
        try:
            search.put_hits(region, self.cap, count, stream)
        except _native.NativeError as e:
            if e.code != _native.MP_E_CAP:
                raise
            self._need = max(self._need, e.need)
            return False
        return True

    def settle(self) -> bool:
        """Collective, after every rank synchronised the streams of its puts: if any rank's put
        did not fit, regrow the regions to twice the largest need and put every slot's last run
        again (the handles must still hold those runs).  True when a regrow happened."""
        import torch
        import torch.distributed as dist
        needs = [None] * self.world
        dist.all_gather_object(needs, int(self._need), group=self.group)
        if max(needs) <= self.cap:
            return False
        self.close()                                # every rank unmaps the old buffers ...
        dist.barrier(group=self.group)              # ... before rank 0 frees them
        self._buf = self._cnt = None
        self.cap = 2 * max(needs)
        self._need = 0
        self._map()
        for slot, (search, stream) in sorted(self._last.items()):
            self.put(search, stream, slot)
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        self.regrowths += 1
        return True

    def hits(self, seq_shifts=None, slot: int = 0):
        """Rank 0: the rank-ordered hit bytes of `slot` (a torch uint8 tensor on its device),
        rank r's sequence indices plus seq_shifts[r] (contig shards)."""
        import torch
        n = self.counts(slot)
        parts = []
        for r in range(self.world):
            at = (slot * self.world + r) * self.cap
            part = self._buf[at * HIT_BYTES:(at + n[r]) * HIT_BYTES].clone()
            if seq_shifts and seq_shifts[r] and n[r]:
                # mp_hit = {u64 pos1, u64 pos2, u32 seq, u32 rec}: seq is int32 word 4 of 6
                part.view(torch.int32).view(n[r], HIT_BYTES // 4)[:, 4] += int(seq_shifts[r])
            parts.append(part)
        return torch.cat(parts)

    def counts(self, slot: int = 0):
        if self._cnt is None:
            return None
        return self._cnt[slot * self.world:(slot + 1) * self.world].cpu().tolist()

    def close(self):
        from . import _native
        for p in self._opened:
            _native.ipc_close(p)
        self._opened = []


def gather_hits(local, n_local: int, group=None, dst: int = 0, seq_base: int = 0) -> Optional[object]:
    """Gather per-rank hit byte buffers (torch uint8 tensors) to rank ``dst``.

    ``local`` holds at least n_local * 24 bytes.  ``seq_base`` (contig sharding)
    is added to every hit's record index first, in place.  Returns the
    concatenated tensor on rank ``dst`` (rank order), None elsewhere.
    """
    import torch
    import torch.distributed as dist

    if seq_base and n_local:
        # mp_hit = {u64 pos1, u64 pos2, u32 seq, u32 rec}: seq is int32 word 4 of 6
        words = local[:n_local * HIT_BYTES].view(torch.int32).view(n_local, HIT_BYTES // 4)
        words[:, 4] += seq_base

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = local.device
    cnt = torch.tensor([n_local], dtype=torch.int64, device=dev)
    counts = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, cnt, group=group)
    counts = [int(c) for c in counts.cpu().tolist()]  # one device-to-host read
    if rank == dst:
        total = sum(counts)
        out = torch.empty(max(total, 1) * HIT_BYTES, dtype=torch.uint8, device=dev)
        ops = []
        off = 0
        for r, c in enumerate(counts):
            if c == 0:
                off += c
                continue
            view = out[off * HIT_BYTES:(off + c) * HIT_BYTES]
            if r == rank:
                view.copy_(local[:c * HIT_BYTES])
            else:
                ops.append(dist.P2POp(dist.irecv, view, r, group=group))
            off += c
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        return out[:total * HIT_BYTES]
    if n_local:
        op = dist.P2POp(dist.isend, local[:n_local * HIT_BYTES].contiguous(), dst, group=group)
        for w in dist.batch_isend_irecv([op]):
            w.wait()
    return None


def as_hits(buf) -> np.ndarray:
    """uint8 tensor / array of packed mp_hit records -> structured numpy array."""
    from ._native import HIT_DTYPE
    arr = buf.cpu().numpy() if hasattr(buf, "cpu") else np.asarray(buf)
    return np.frombuffer(arr.tobytes(), dtype=HIT_DTYPE)
