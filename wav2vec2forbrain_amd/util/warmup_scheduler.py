"""Mirrors reference src/util/warmup_scheduler.py:5-57 (2-group LambdaLR warmup, stepped per epoch)."""
from torch.optim.lr_scheduler import LambdaLR
from torch.optim.optimizer import Optimizer


def get_2module_warmup_scheduler(optimizer: Optimizer, module1_baselr: float, module2_warmup_start_step: int,
                                 module2_warmup_steps: int, module2_target_lr: float,
                                 adjust_module1_lr_to_module2_postwarmup_lr: bool):
    def module2_lr(step: int):
        if step < module2_warmup_start_step:
            return 0.0
        return min(1.0, (step - module2_warmup_start_step) / module2_warmup_steps if module2_warmup_steps > 0 else 1.0)

    def module1_lr(step: int):
        if not adjust_module1_lr_to_module2_postwarmup_lr or module2_target_lr is None or module2_target_lr == 0.0:
            return 1.0
        if step < module2_warmup_start_step:
            return 1.0
        target_factor = module2_target_lr / module1_baselr
        if step >= module2_warmup_start_step + module2_warmup_steps:
            return target_factor
        return 1.0 + (target_factor - 1.0) * (step - module2_warmup_start_step) / module2_warmup_steps

    return LambdaLR(optimizer, lr_lambda=[module1_lr, module2_lr])
