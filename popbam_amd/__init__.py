"""popbam_amd -- MI355X-native hot path of POPBAM 0.3 (per-site consensus call + per-window
population-genetics statistics) behind a C-ABI (include/popbam_gpu.h).

  options  host mirror of the reference CLI / region / @RG sample model
  engine   one `popbam <cmd>` run on the GPU (pbg_run)
  _lib     ctypes binding of libpopbam_gpu.so (built in-tree from csrc/)
"""
from . import options  # noqa: F401

__all__ = ["options", "engine", "_lib"]
