"""bn_relu_maxpool_fwd at the ResNet-50 stem shape (256 x 64 x 112 x 112 -> 56 x 56, bf16), us per
call, outputs and window indices checked against a PyTorch reference once; FLUXMPI_POOL_GENERIC=1
selects the runtime-window kernel. One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fluxmpi_amd.ops import _ext  # noqa: E402
from fluxmpi_amd.ops.multi_tensor import DTYPE_CODE  # noqa: E402

C = _ext.get(required=True)
n, ch, h, w = 256, 64, 112, 112
x = torch.randn(n, h, w, ch, device="cuda").bfloat16()
scale = torch.rand(ch, device="cuda") + 0.5
shift = torch.randn(ch, device="cuda") * 0.1
y = torch.empty(n, 56, 56, ch, device="cuda", dtype=torch.bfloat16)
idx = torch.empty(n * 56 * 56 * ch, device="cuda", dtype=torch.uint8)
s = torch.cuda.current_stream().cuda_stream
f = lambda: C.bn_relu_maxpool_fwd(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), y.data_ptr(), idx.data_ptr(),  # noqa: E731
                                  n, h, w, ch, 3, 2, 1, DTYPE_CODE[torch.bfloat16], s)
f()
z = torch.relu(x.float() * scale + shift).permute(0, 3, 1, 2)
ref = torch.nn.functional.max_pool2d(z, 3, 2, 1).permute(0, 2, 3, 1)
err = float((y.float() - ref).abs().max())
for _ in range(3):
    f()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = float("inf")
for _ in range(3):
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
print(json.dumps({"generic": bool(os.environ.get("FLUXMPI_POOL_GENERIC")), "us": round(best, 1), "max_abs_err": err,
                  "tbs_unique": round((x.numel() * 2 + y.numel() * 2 + idx.numel()) / best / 1e6, 2)}), flush=True)
