"""DDP / FSDP plugins (reference ``thunder/plugins/distributed.py``), incl. the hybrid 2-D mesh.

``FSDP(process_group=mesh)`` with a ``DeviceMesh`` whose dims are ``("ddp", "fsdp")`` shards
parameters inside each ``fsdp`` group and all-reduces the gradient shards across ``ddp``
replicas (hybrid sharding: the natural layout for an MI355X node, fsdp = the 8 GPUs of a node
on xGMI, ddp = across nodes).
"""
from __future__ import annotations

import torch.distributed as tdist

from ..core.recipe import Plugin
from ..distributed import copy_default_process_group


class DDP(Plugin):
    def __init__(self, bucket_size_in_mb: float = 256.0, broadcast_from: int | None = None, process_group=None):
        self.bucket_size_in_mb = bucket_size_in_mb
        self.broadcast_from = broadcast_from
        self.process_group = process_group

    def setup_transforms(self):
        from ..distributed.transforms import DDPTransform

        pg = self.process_group if self.process_group is not None else copy_default_process_group()
        return [DDPTransform(process_group=pg, bucket_size_in_mb=self.bucket_size_in_mb,
                             broadcast_from=self.broadcast_from)]


class FSDP(Plugin):
    def __init__(self, device=None, broadcast_from: int | None = None, sharding_strategy=None, bucketing_strategy=None,
                 move_state_dict_to_cpu: bool = False, ddp_bucket_size_in_mb: float = 256.0, process_group=None):
        self.device = device
        self.broadcast_from = broadcast_from
        self.sharding_strategy = sharding_strategy
        self.bucketing_strategy = bucketing_strategy
        self.move_state_dict_to_cpu = move_state_dict_to_cpu
        self.ddp_bucket_size_in_mb = ddp_bucket_size_in_mb
        self.process_group = process_group

    def setup_transforms(self):
        from ..distributed.transforms import FSDPTransform, FSDPType, FSDPBucketingStrategy
        from ..transforms.materialization import MaterializationTransform

        pg = self.process_group
        replicate = None
        dims = getattr(pg, "mesh_dim_names", None)
        if dims is not None:
            if tuple(dims) != ("ddp", "fsdp"):
                raise ValueError(f"FSDP plugin expects a DeviceMesh with dims ('ddp', 'fsdp'), got {dims}")
            replicate = pg["ddp"].get_group()
            pg = pg["fsdp"].get_group()
        elif pg is None:
            pg = copy_default_process_group()
        fsdp = FSDPTransform(process_group=pg, sharding_strategy=self.sharding_strategy or FSDPType.ZERO2,
                             bucketing_strategy=self.bucketing_strategy or FSDPBucketingStrategy.NONE,
                             broadcast_from=self.broadcast_from, device=self.device,
                             replicate_process_group=replicate)
        return [fsdp, MaterializationTransform(fsdp, device=self.device)]
