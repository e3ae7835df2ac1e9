"""Training-progress logger with the reference's method names (utils/logger.py).

tensorboard is not a dependency here: ``set_logger_level(use_logger=True)`` writes scalars to
a tensorboard SummaryWriter when one is importable and otherwise to an in-memory list;
``use_logger=False`` gives the printing logger, ``quiet=True`` one that records silently.
"""
from __future__ import annotations

import time

logger = None


class LoggerBase:
    def __init__(self, debug=True):
        self.debug = debug

    def log_scalar(self, category, value, epoch_iteration=None):
        raise NotImplementedError

    def log_scalars(self, category, value, global_step=None):
        raise NotImplementedError

    def log_histogram(self, category, values):
        raise NotImplementedError

    def finalize(self):
        pass

    def log_progress(self, progress):
        tid = progress.get("task") + 1
        self.log_scalar(f"Rewards/Episode/Task_{tid}", progress.get("ep_reward"), progress.get("episodes"))
        self.log_scalar("GPI_%/Task", progress.get("GPI%"), tid)
        self.log_scalar(f"Rewards/Step/Task_{tid}", progress.get("reward"), progress.get("steps"))
        self.log_scalar(f"W_Error/Step/Task_{tid}", progress.get("w_err"), progress.get("steps"))

    def log_target_error_progress(self, progress):
        tid, steps = progress.get("task") + 1, progress.get("steps")
        self.log_scalar(f"Target_Tasks/W_Error/Ev_Steps/task_{tid}", progress.get("w_error"), steps)
        self.log_scalar(f"Target_Tasks/Rewards/Ev_Steps/task_{tid}", progress.get("reward"), steps)
        for key, tag in (("phi_loss", "Phi_Loss"), ("psi_loss", "Psi_Loss"),
                         ("target_loss_coefficient", "Losses/Coefficients")):
            if progress.get(key) is not None:
                self.log_scalar(f"Target_Tasks/{tag}/Ev_Steps/task_{tid}", progress.get(key), steps)

    def log_tasks_performance(self, performances):
        for task, perf in enumerate(performances):
            self.log_scalar("Overall_Performance/Task", perf, task + 1)

    def log_average_reward(self, progress, training_steps):
        self.log_scalar("Average_Reward/timesteps", progress, training_steps)

    def log_accumulative_reward(self, progress, training_steps):
        self.log_scalar("Accumulative_Reward/timesteps", progress, training_steps)

    def log_phi_loss(self, progress, training_steps):
        self.log_scalar("Losses/Phi_Loss/timesteps", progress, training_steps)

    def log_psi_loss(self, progress, training_steps):
        self.log_scalar("Losses/Psi_Loss/timesteps", progress, training_steps)

    def log_total_loss(self, progress, training_steps):
        self.log_scalar("Losses/Total_Loss/timesteps", progress, training_steps)

    def log_loss_coefficient(self, progress, training_steps):
        if len(progress) > 1:
            self.log_scalar("Losses/Coefficients_L1/timesteps", progress[0], training_steps)
            self.log_scalar("Losses/Coefficients_L2/timesteps", progress[1], training_steps)
        else:
            self.log_scalar("Losses/Coefficients/timesteps", progress[0], training_steps)

    def log_losses(self, total_loss, psi_loss, phi_loss, loss_coefficient, training_steps):
        self.log_phi_loss(phi_loss, training_steps)
        self.log_psi_loss(psi_loss, training_steps)
        self.log_total_loss(total_loss, training_steps)
        self.log_loss_coefficient(loss_coefficient, training_steps)

    def log_omegas_learning_rate(self, learning_rate, task_id, total_steps):
        self.log_scalar(f"Target_Tasks/Omegas_Learning_Rate/Ev_Steps/task_{task_id + 1}", learning_rate, total_steps)

    def log_source_performance(self, task_id, reward, training_steps):
        self.log_scalar(f"Source_Tasks/Rewards/task_{task_id + 1}", reward, training_steps)


class Logger(LoggerBase):
    """Scalars to tensorboard when available, else kept in ``self.records``."""

    def __init__(self, debug=True):
        super().__init__(debug)
        self.records = []
        try:
            from torch.utils.tensorboard import SummaryWriter

            self.writer = SummaryWriter("data/dynamics_sfdqn_run_%s" % time.strftime("%d_%m_%Y_%H_%M_%S"))
        except Exception:
            self.writer = None

    def log_scalar(self, category, value, epoch_iteration=None):
        if self.writer is not None:
            self.writer.add_scalar(category, value, epoch_iteration)
        else:
            self.records.append((category, value, epoch_iteration))

    def log_scalars(self, category, value, global_step=None):
        if self.writer is not None:
            self.writer.add_scalars(category, value, global_step)
        else:
            self.records.append((category, value, global_step))

    def log_histogram(self, category, values):
        if self.writer is not None:
            self.writer.add_histogram(category, values)

    def finalize(self):
        if self.writer is not None:
            self.writer.flush()
            self.writer.close()


class MockLogger(LoggerBase):
    def __init__(self, debug=True, quiet=False):
        super().__init__(debug)
        self.quiet = quiet

    def log_scalar(self, category, value, epoch_iteration=None):
        if not self.quiet:
            print(f"{category} Value: {value} Epoch: {epoch_iteration}")

    def log_scalars(self, category, value, global_step=None):
        if not self.quiet:
            print(f"{category} Value: {value} Epoch: {global_step}")

    def log_histogram(self, category, values):
        if not self.quiet:
            print(f"{category} Values: {values}")


def set_logger_level(use_logger=False, quiet=False):
    global logger
    if logger is None:
        logger = Logger() if use_logger else MockLogger(quiet=quiet)
    return logger


def get_logger_level():
    return logger
