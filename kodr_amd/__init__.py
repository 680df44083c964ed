"""kodr_amd -- MI355X-native (gfx950) RLNC engine with itzmeanjan/kodr's API.

Layout:
  csrc/            HIP kernel (gf_kernels.hip), C ABI (capi.cpp, capi_decoder.cpp), host mirror of
                   kodr's decoder state (decoder_core.cpp)
  libkodr_rlnc.so  built in-tree by build.sh; the only compute path
  full, systematic, kodr_internals, errors
                   Python mirror of kodr's Go packages over the C ABI
"""
from . import errors  # noqa: F401
from ._lib import LIB_PATH, LibraryMissing, lib  # noqa: F401

__version__ = "0.1.0"


def build(verbose=False):
    """Compile libkodr_rlnc.so for gfx950 in-tree (hipcc; no GPU needed)."""
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run(["bash", os.path.join(here, "build.sh")], capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("kodr_amd build failed:\n" + (r.stdout or "") + (r.stderr or ""))
