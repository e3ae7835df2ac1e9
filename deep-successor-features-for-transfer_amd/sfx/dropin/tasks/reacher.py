"""Reacher tasks (tasks/reacher.py): the pybullet physics stays on the host.

pybullet / pybulletgym are not installed in this image; constructing ``Reacher`` raises with
that message.  ``tasks.synthetic.SyntheticReacher`` has the same interface and shapes.
"""
from tasks.task import Task


class Reacher(Task):
    def __init__(self, target_positions, task_index, include_target_in_state=False):
        try:
            import pybulletgym  # noqa: F401
        except ImportError as e:
            raise ImportError("tasks.reacher.Reacher needs pybullet + pybulletgym (not installed here); "
                              "use tasks.synthetic.SyntheticReacher for a Reacher-shaped task") from e
        raise NotImplementedError("the pybullet Reacher env is outside sfx's scope (host env, DESIGN.md §9)")
