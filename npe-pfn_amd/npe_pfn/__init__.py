"""MI355X-native NPE-PFN.

Same public names as the reference package (npe_pfn/__init__.py:1-12), so
``from npe_pfn import TabPFN_Based_NPE_PFN, run_tsnpe_pfn`` keeps working with
this directory (``npe-pfn_amd``) on ``sys.path``.  The TabPFN forward runs in
the HIP engine ``npe_pfn/_lib/libnpfn.so`` (C-ABI: include/npfn.h).
"""

from npe_pfn.npe_pfn import NPE_PFN_Core, TabPFN_Based_NPE_PFN
from npe_pfn.tsnpe_pfn import run_tsnpe_pfn

__all__ = [
    "NPE_PFN_Core",
    "TabPFN_Based_NPE_PFN",
    "run_tsnpe_pfn",
]
