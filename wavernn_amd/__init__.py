"""wavernn_amd — MI355X-native WaveRNN generation path.

Drop-in for the reference's `models.fatchord_version.WaveRNN` (constructor, state_dict,
load/save, generate()), with the autoregressive sample loop running as one persistent
CDNA4 kernel behind the C-ABI in include/wavernn_amd.h.  Submodules import lazily so that
building/inspecting the package never needs a GPU."""
__version__ = "0.1.0"


def __getattr__(name):
    if name == "WaveRNN":
        from .fatchord_version import WaveRNN
        return WaveRNN
    if name == "FatchordLoop":
        from .loop import FatchordLoop
        return FatchordLoop
    raise AttributeError(name)
