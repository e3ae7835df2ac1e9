"""MDP interface the agents drive (tasks/task.py:2-127)."""


class Task:
    def clone(self):
        raise NotImplementedError

    def initialize(self):
        raise NotImplementedError

    def action_count(self):
        raise NotImplementedError

    def transition(self, action):
        """-> (next state, reward, terminal)"""
        raise NotImplementedError

    def encode(self, state):
        raise NotImplementedError

    def encode_dim(self):
        raise NotImplementedError

    def features(self, state, action, next_state):
        raise NotImplementedError

    def feature_dim(self):
        raise NotImplementedError

    def get_w(self):
        raise NotImplementedError
