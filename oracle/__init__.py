"""ORACLE -- CPU restatement of the reference path. Test infrastructure only.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Never imported by the product package (npe-pfn_amd/).
"""
