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
