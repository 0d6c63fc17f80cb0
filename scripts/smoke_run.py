"""Run __graft_entry__.smoke() in its own process (GPU scripts)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
print("smoke ok")
