"""Full-pool integrity scan sharded across GPUs (BASELINE config 5).

One process per GPU.  Chunk files are sharded by contiguous chunk-index range;
each rank hashes its own files on its own GPU with no data-path collective.  The
only exchange is the per-copyset digest: CopysetNode::GetHash
(src/chunkserver/copyset_node.cpp:925-975) is an ORDERED chain over files in
std::sort name order, but in the linear GF(2) domain each file contributes
shift(V(file), bytes after it in that order), so every rank computes order-free
XOR partials for the files it holds and one all_gather of 4 B per copyset per
rank (RCCL over xGMI on GPUs, gloo on CPU) finishes it.  A commutative XOR is
not an RCCL reduction op, hence all_gather + local XOR rather than all_reduce.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence

from .scan import chunk_file_name, copyset_after_bytes


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous chunk-index range [lo, hi) of `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


@dataclass
class CopysetLayout:
    """Which copyset each chunk file belongs to and its digest shift."""
    names: List[str]
    group: List[int]          # copyset index per file
    after_bytes: List[int]    # bytes of the same copyset sorting after the file
    n_groups: int


def copyset_layout(chunk_ids: Sequence[int], copyset_of: Sequence[int], file_bytes: Sequence[int]) -> CopysetLayout:
    """Geometry of the whole pool (every rank computes the same layout)."""
    names = [chunk_file_name(c) for c in chunk_ids]
    groups = sorted(set(copyset_of))
    gidx = {g: i for i, g in enumerate(groups)}
    group = [gidx[g] for g in copyset_of]
    after = [0] * len(names)
    members: Dict[int, List[int]] = {}
    for i, g in enumerate(group):
        members.setdefault(g, []).append(i)
    for g, mem in members.items():
        for i, a in zip(mem, copyset_after_bytes([names[i] for i in mem], [file_bytes[i] for i in mem])):
            after[i] = a
    return CopysetLayout(names, group, after, len(groups))


def reduce_digests(partial, dist, group=None):
    """XOR-reduce per-copyset partials (int32 tensor [n_groups]) over all ranks:
    all_gather_into_tensor (RCCL/gloo) then a local XOR fold.  Returns the full
    digests on every rank."""
    import torch
    world = dist.get_world_size(group)
    if world == 1:
        return partial
    dev = partial.device
    if dist.get_backend(group) == "gloo" and partial.is_cuda:
        partial = partial.cpu()  # gloo moves host tensors; RCCL works on device tensors
    gathered = torch.empty(world * partial.numel(), dtype=partial.dtype, device=partial.device)
    dist.all_gather_into_tensor(gathered, partial.contiguous(), group=group)
    g = gathered.view(world, -1)
    out = g[0].clone()
    for r in range(1, world):
        out.bitwise_xor_(g[r])
    return out.to(dev)


def digests_as_hash_strings(digests) -> List[str]:
    """Per-copyset digests -> GetCopysetStatus(queryhash) strings (std::to_string(uint32))."""
    return [str(int(x) & 0xFFFFFFFF) for x in digests.detach().cpu().tolist()]
