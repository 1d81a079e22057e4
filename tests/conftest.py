import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libis3d_amd.so on the GPU)")


def pytest_sessionstart(session):
    # torch bundles its own HIP runtime (libamdhip64.so) beside the system one libis3d_amd.so links
    # (libamdhip64.so.7): torch's initialises only if it comes first, so a GPU session starts it before any test
    # loads the engine (a module run alone, e.g. test_gpu_north_star.py, otherwise failed in torch's cuda init)
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.device_count() > 0:
        torch.cuda.init()
