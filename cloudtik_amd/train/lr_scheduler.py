"""Learning-rate schedules used by the reference workloads.

* ``LinearWarmupPolyDecayScheduler`` -- BERT-large pretraining
  (bert_large/training/schedulers.py:52; start_warmup_steps / warmup_steps / total_steps /
  end_learning_rate / degree, offset_step semantics preserved).
* ``LinearWarmUpScheduler`` -- schedulers.py LinearWarmUpScheduler.
* ``StepDecayScheduler`` -- ResNet-50 (lr * 0.1 every 30 epochs, common/main.py).

They write ``param_group['lr']`` on the host; the fused optimizers copy it into their
device-side hyper-parameter array at ``step()`` (no per-step sync).
"""
from __future__ import annotations


class _Sched:
    def __init__(self, optimizer):
        self.optimizer = optimizer
        self.base_lrs = [g["lr"] for g in optimizer.param_groups]
        self.last_epoch = 0

    def _set(self, lrs):
        for g, lr in zip(self.optimizer.param_groups, lrs):
            g["lr"] = lr

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"last_epoch": self.last_epoch, "base_lrs": self.base_lrs}

    def load_state_dict(self, sd):
        self.last_epoch = sd["last_epoch"]
        self.base_lrs = sd["base_lrs"]


class LinearWarmupPolyDecayScheduler(_Sched):
    def __init__(self, optimizer, start_warmup_steps, warmup_steps, total_steps,
                 end_learning_rate=0.0, degree=1.0):
        super().__init__(optimizer)
        self.num_warmup_updates = warmup_steps
        self.start_warmup_steps = start_warmup_steps
        self.total_steps = total_steps
        self.end_learning_rate = end_learning_rate
        self.degree = degree
        self.offset_step = int(start_warmup_steps == 0)
        self.last_epoch = 1
        self._set(self.get_lr())

    def get_lr(self):
        mod_step = self.last_epoch - self.offset_step - self.start_warmup_steps
        cond = float(mod_step < self.num_warmup_updates)
        progress = cond * (mod_step / (self.num_warmup_updates + 1e-6)) + \
            (1.0 - cond) * min((self.last_epoch - self.offset_step) / self.total_steps, 1)
        base = self.base_lrs[0]
        lr = cond * (base * progress) + (1.0 - cond) * (
            (base - self.end_learning_rate) * (1 - progress) ** self.degree + self.end_learning_rate)
        return [lr for _ in self.base_lrs]

    def step(self):
        self.last_epoch += 1
        self._set(self.get_lr())


class LinearWarmUpScheduler(_Sched):
    def __init__(self, optimizer, warmup, total_steps):
        super().__init__(optimizer)
        self.warmup, self.total_steps = warmup, total_steps

    def get_lr(self):
        progress = self.last_epoch / self.total_steps
        if progress < self.warmup:
            return [b * progress / self.warmup for b in self.base_lrs]
        return [b * max((progress - 1.0) / (self.warmup - 1.0), 0.0) for b in self.base_lrs]

    def step(self):
        self.last_epoch += 1
        self._set(self.get_lr())


class StepDecayScheduler(_Sched):
    def __init__(self, optimizer, step_size, gamma=0.1, warmup_steps=0):
        super().__init__(optimizer)
        self.step_size, self.gamma, self.warmup_steps = step_size, gamma, warmup_steps

    def get_lr(self):
        e = self.last_epoch
        if self.warmup_steps and e < self.warmup_steps:
            return [b * (e + 1) / self.warmup_steps for b in self.base_lrs]
        return [b * (self.gamma ** (e // self.step_size)) for b in self.base_lrs]

    def step(self):
        self.last_epoch += 1
        self._set(self.get_lr())


class WarmupMultiStepScheduler(_Sched):
    """Mask R-CNN / SSD schedule (maskrcnn_benchmark solver/lr_scheduler.py WarmupMultiStepLR):
    linear warm-up from ``warmup_factor`` x lr over ``warmup_steps``, then x``gamma`` at
    each milestone step."""

    def __init__(self, optimizer, milestones, gamma=0.1, warmup_factor=1.0 / 3, warmup_steps=500):
        super().__init__(optimizer)
        self.milestones, self.gamma = sorted(int(m) for m in milestones), gamma
        self.warmup_factor, self.warmup_steps = warmup_factor, warmup_steps
        self._set(self.get_lr())

    def get_lr(self):
        e = self.last_epoch
        f = 1.0
        if e < self.warmup_steps:
            a = e / max(1, self.warmup_steps)
            f = self.warmup_factor * (1 - a) + a
        decay = self.gamma ** sum(1 for m in self.milestones if e >= m)
        return [b * f * decay for b in self.base_lrs]

    def step(self):
        self.last_epoch += 1
        self._set(self.get_lr())
