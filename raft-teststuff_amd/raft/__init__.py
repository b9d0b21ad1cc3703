"""MI355X-native RAFT frequency-domain response solve (drop-in for the reference's
`import raft; raft.Model(design)` / `raft.runRAFT(file)` on the hot path).  See DESIGN.md."""
from .model import Model, runRAFT, runRAFTFarm
from .fowt import FOWT
from .member import Member

__all__ = ["Model", "FOWT", "Member", "runRAFT", "runRAFTFarm"]
