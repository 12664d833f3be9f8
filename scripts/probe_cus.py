"""Probe: the device's compute-unit count and clocks as this process sees them (box-to-box
variance of one-round kernels such as k_dcn_bwd_weight3).  GPU box only."""
import json
import torch
p = torch.cuda.get_device_properties(0)
print(json.dumps({'name': p.name, 'multi_processor_count': p.multi_processor_count,
                  'gcn_arch': getattr(p, 'gcnArchName', None), 'total_memory_gb': round(p.total_memory / 2**30, 1),
                  'l2_cache_size': getattr(p, 'L2_cache_size', None)}))
