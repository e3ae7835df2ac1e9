"""The single-file TSF-DQN (tsfdqn.py: ReplayBuffer, DeepTSF, TSFDQN) on libsfx.

tsfdqn.py:10-1011 is tsfdqn_nf.py with g_i = nn.Linear(n_s, G) (no planar flows) -- i.e. the
sequential TSF stack of agents.tsfdqn_sequential / features.deep_sequential_tsf here, whose
update (tsfdqn.py:588-709) runs as one sfx_tsf_update call per env step.
"""
from __future__ import annotations

from agents.buffer_tsf_sequential import ReplayBuffer  # noqa: F401  (tsfdqn.py:10-90)
from agents.tsfdqn_sequential import TSFDQN  # noqa: F401  (tsfdqn.py:329-1011)
from tsfdqn_nf import DeepTSF  # noqa: F401  (tsfdqn.py:93-326: use_true_reward positional)
