"""Cross-rank gather of decoded batches.

Ranks decode disjoint shards of the sample index space; when one rank needs every
decision (e.g. to write them out), each rank bit-packs its shard on the device
(`DecoderGPU.pack_decisions_dev`, one record of 2 ceil(n/8) + 1 bytes per syndrome)
and the records are gathered to rank 0 over RCCL (xGMI) -- 8x fewer bytes than the
0/1 byte arrays.  This is not part of the decode step: syndromes are independent and
the decode needs no exchange."""
import numpy as np


def gather_records(packed, dst=0, group=None):
    """Gathers equally sized [B, R] uint8 record tensors of every rank to `dst`: returns the
    [world * B, R] tensor (rank order = sample order) on dst, None elsewhere.  Without an
    initialised process group (one process) it returns `packed` itself.

    The collective follows from the backend alone, the same on every rank (no fallback that
    could leave ranks in different collectives): gloo gathers host copies; nccl (RCCL over
    xGMI) gathers the device tensors straight into the output's row blocks.  Only dst
    allocates the output."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return packed
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    root = rank == dst
    if dist.get_backend(group) == "gloo":
        src = packed.detach().cpu().contiguous()
        parts = [torch.empty_like(src) for _ in range(world)] if root else None
        dist.gather(src, gather_list=parts, dst=dst, group=group)
        if not root:
            return None
        full = torch.cat(parts)
        return full.to(packed.device) if packed.is_cuda else full
    out = torch.empty((world * packed.shape[0], packed.shape[1]), dtype=packed.dtype,
                      device=packed.device) if root else None
    dist.gather(packed.contiguous(), gather_list=list(out.chunk(world)) if root else None, dst=dst, group=group)
    return out


def _gather_into(packed, out, dst, group):
    """gather_records into a preallocated root output (`out`: [world * B, R], a device tensor under
    RCCL, a host tensor under gloo; ignored off the root).  Same collective choice as gather_records."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    root = dist.get_rank(group) == dst
    src = packed if dist.get_backend(group) != "gloo" else packed.detach().cpu()
    dist.gather(src.contiguous(), gather_list=list(out.chunk(world)) if root else None, dst=dst, group=group)


class GatherPipeline:
    """Decode and gather overlapped: every rank decodes step k + 1 into one of two
    record buffers while step k's records, in the other, are gathered to `dst` -- the decode on the
    caller's (compute) stream, the gather on a communication stream, ordered by events only:

        compute: [wait gather(k - 1) freed buf (k+1)%2] decode(k + 1) -> done[(k+1)%2]
        comm:    [wait done[k%2]] gather(buf k%2) -> root out[k%2] -> sink(k) -> freed[k%2]

    Under RCCL (backend "nccl") both run asynchronously on the device (the gather's RCCL stream waits on
    the communication stream, which waits on the decode's event); under gloo the host copy and the
    host-side gather of step k run while the device decodes step k + 1, already enqueued.  Only the
    root keeps gathered outputs (two, reused alternately).  The reference's counterpart is the
    sample-parallel loop of QEC_LDPC/DecoderCPU.h:419-438, whose results stay in one process."""

    def __init__(self, record_shape, device, dst=0, group=None):
        import torch
        import torch.distributed as dist
        self.device = device
        self.dst, self.group = dst, group
        self.dist = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.root = (dist.get_rank(group) if dist.is_initialized() else 0) == dst
        self.gloo = dist.is_initialized() and dist.get_backend(group) == "gloo"
        B, R = record_shape
        self.bufs = [torch.empty((B, R), dtype=torch.uint8, device=device) for _ in range(2)]
        odev = torch.device("cpu") if self.gloo else device
        self.outs = [torch.empty((self.world * B, R), dtype=torch.uint8, device=odev) for _ in range(2)] \
            if self.root else [None, None]
        self.comm = torch.cuda.Stream(device)
        self.done = [torch.cuda.Event() for _ in range(2)]
        self.freed = [None, None]

    def _decode(self, decode, k, compute):
        j = k % 2
        if self.freed[j] is not None:
            compute.wait_event(self.freed[j])  # step k - 2's gather has read this buffer
        decode(k, self.bufs[j], compute)
        self.done[j].record(compute)

    def _gather(self, k, sink):
        import torch
        j = k % 2
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.done[j])
            if not self.dist:  # one process: the "gather" is a copy into the output
                self.outs[j].copy_(self.bufs[j])
            else:
                _gather_into(self.bufs[j], self.outs[j], self.dst, self.group)
            if sink is not None and self.root:
                sink(k, self.outs[j])  # on the communication stream: ordered after the gather
            ev = torch.cuda.Event()
            ev.record(self.comm)
            self.freed[j] = ev

    def run(self, decode, steps, sink=None):
        """decode(k, rec, stream) enqueues step k's decode into rec on stream; sink(k, out) (root only)
        sees step k's gathered [world * B, R] records on the communication stream (copy or clone what
        must outlive the next-but-one step).  Returns after the last gather completed on this rank."""
        import torch
        compute = torch.cuda.current_stream(self.device)
        if steps <= 0:
            return
        self._decode(decode, 0, compute)
        for k in range(steps):
            if k + 1 < steps:
                self._decode(decode, k + 1, compute)
            self._gather(k, sink)
        compute.wait_stream(self.comm)
        torch.cuda.synchronize(self.device)


def unpack_records(records, n):
    """Host inverse of qec_pack_decisions_dev: [B, 2 ceil(n/8) + 1] -> (eX, eZ, flags)."""
    records = np.asarray(records, dtype=np.uint8)
    nb = (n + 7) // 8
    eX = np.unpackbits(records[:, :nb], axis=1, bitorder="little")[:, :n]
    eZ = np.unpackbits(records[:, nb:2 * nb], axis=1, bitorder="little")[:, :n]
    return eX, eZ, records[:, 2 * nb].copy()


def pack_records(eX, eZ, flags):
    """Host equivalent of qec_pack_decisions_dev (used to check it and on CPU-only ranks)."""
    return np.concatenate([np.packbits(np.asarray(eX, np.uint8) & 1, axis=1, bitorder="little"),
                           np.packbits(np.asarray(eZ, np.uint8) & 1, axis=1, bitorder="little"),
                           np.asarray(flags, np.uint8).reshape(-1, 1)], axis=1)
