"""Compare wave_accumulate's per-row normal equations with torch (GPU debug probe)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from oryx_amd import native
from oryx_amd.ops import als as als_ops
lib = native.require_kernels()
dev = torch.device("cuda")
for kp in (16, 64, 112):
    for n in (5, 32, 45, 100):
        g = torch.Generator().manual_seed(kp + n)
        cols = torch.randperm(500, generator=g)[:n].int()
        vals = (torch.randint(1, 10, (n,), generator=g).float() * 0.5)
        row_ptr = torch.tensor([0, n], dtype=torch.int64)
        Y = (torch.randn(500, kp, generator=g) * 0.3).bfloat16()
        out = torch.zeros(kp * kp + kp + 1, device=dev)
        # keep the device copies alive until the kernel has run
        d_rp, d_c, d_v, d_y = row_ptr.to(dev), cols.to(dev), vals.to(dev), Y.to(dev)
        rc = lib.oryx_als_debug_gram(d_rp.data_ptr(), d_c.data_ptr(), d_v.data_ptr(),
                                     d_y.data_ptr(), kp, 1.0, 1, 0, n, out.data_ptr(),
                                     native.stream_ptr(dev))
        torch.cuda.synchronize()
        o = out.cpu()
        y = Y.float()[cols.long()]
        wa = vals.abs()
        A = (y * wa[:, None]).t() @ y
        b = ((1 + wa)[:, None] * y).sum(0)
        gA = o[:kp * kp].view(kp, kp)
        gb = o[kp * kp:kp * kp + kp]
        print(kp, n, "A err %.3g (scale %.3g)" % ((gA - A).abs().max(), A.abs().max()),
              "b err %.3g (scale %.3g)" % ((gb - b).abs().max(), b.abs().max()),
              "cnt", float(o[-1]))
        if (gA - A).abs().max() > 0.05 * A.abs().max():
            print(" A diag got", gA.diag()[:8].tolist())
            print(" A diag ref", A.diag()[:8].tolist())
            print(" A row0 got", gA[0, :8].tolist())
            print(" A row0 ref", A[0, :8].tolist())
            print(" b got", gb[:8].tolist())
            print(" b ref", b[:8].tolist())
