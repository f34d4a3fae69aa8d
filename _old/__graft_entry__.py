"""Driver hooks: ``build()`` compiles every HIP extension for gfx950 and imports the
package; ``smoke()`` runs one tiny forward+backward of the flagship model on cuda:0."""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def build() -> None:
    os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    import build as _b
    _b.build()
    import ddl_amd  # noqa: F401
    from ddl_amd.ops import native
    assert native.available(), native.error()
    from ddl_amd.parallel import roles, comm, sharding  # noqa: F401


def smoke() -> None:
    import torch
    from ddl_amd.ops import native
    from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL
    from ddl_amd.models.mnist_cnn import init_params_
    from ddl_amd.models.hip_engine import HipEngine
    assert native.available(), native.error()
    dev = torch.device("cuda", 0)
    params = torch.zeros(TOTAL_NUMEL, device=dev)
    init_params_(params, CANON_OFFSETS, 0)
    grads = torch.zeros_like(params)
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=8, graph=False, eval_chunk=8)
    x = torch.rand(8, 784, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    eng.forward_backward(x, y, 0.5, 1)
    torch.cuda.synchronize()
    loss = float(eng.loss())
    assert torch.isfinite(grads).all() and grads.abs().sum() > 0 and loss == loss
    print(f"smoke ok: loss={loss:.4f} |grad|={float(grads.norm()):.4f}")


if __name__ == "__main__":
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "smoke":
        smoke()
