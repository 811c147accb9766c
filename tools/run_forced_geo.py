import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/vaesne-dev_amd"]
import torch
from VAESNe import _lib
geo = tuple(int(v) for v in sys.argv[1].split(","))
_lib.lib.attn_force_geometry(*geo)
import pytest
sys.exit(pytest.main(sys.argv[2:]))
