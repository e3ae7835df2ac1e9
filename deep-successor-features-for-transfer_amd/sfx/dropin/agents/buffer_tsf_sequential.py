"""Uniform experience replay of the TSF sequential scripts (agents/buffer_tsf_sequential.py:8-87,
main_tsfdqn_sequential_torch.py): the same ring and sampling as agents.buffer_sequential."""
from __future__ import annotations

from agents.buffer_sequential import ReplayBuffer  # noqa: F401  (identical interface and semantics)
