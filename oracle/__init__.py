"""CPU oracle package — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. The product path (vfm-vae_amd/) never imports it.
"""
