from .constants import G, P, Q, R, P_BYTES, Q_BYTES, ProductionMode
from .group import (ElementModP, ElementModQ, FixedBase, GroupContext, as_p_array, as_q_array,
                    p_bytes, productionGroup, q_bytes)
from .native import EgError, NativeUnavailable
from .hashing import hash_elems, hexP, hexQ
