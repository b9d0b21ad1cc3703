"""MI355X-native RAFT frequency-domain response solve (drop-in for the reference's
`import raft; raft.Model(design)` on the hot path).  See DESIGN.md."""
from .model import Model
from .fowt import FOWT
from .member import Member

__all__ = ["Model", "FOWT", "Member"]
