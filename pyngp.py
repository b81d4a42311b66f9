"""Top-level `pyngp` name, as imported by the reference drivers (scripts/run.py: `import pyngp as ngp`)."""
from neus2_amd.pyngp import *  # noqa: F401,F403
from neus2_amd.pyngp import Testbed, TestbedMode, nccl_unique_id  # noqa: F401
