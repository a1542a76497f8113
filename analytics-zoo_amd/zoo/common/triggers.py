"""Training triggers (Zs/common/ZooTrigger.scala:26-166, BigDL Trigger [ext]).

A trigger is a predicate over the engine state dict (``epoch``, ``neval``,
``Loss``, ``score``, ``epoch_end``). ``iteration_based`` tells the engine it
may fire inside an epoch.
"""


class Trigger:
    iteration_based = False

    def __call__(self, state):
        raise NotImplementedError

    # BigDL python names
    @staticmethod
    def every_epoch():
        return EveryEpoch()

    @staticmethod
    def several_iteration(n):
        return SeveralIteration(n)

    @staticmethod
    def max_epoch(n):
        return MaxEpoch(n)

    @staticmethod
    def max_iteration(n):
        return MaxIteration(n)


class EveryEpoch(Trigger):
    def __call__(self, state):
        return bool(state.get("epoch_end", False))


class SeveralIteration(Trigger):
    iteration_based = True

    def __init__(self, interval):
        self.interval = int(interval)

    def __call__(self, state):
        it = state["neval"] - 1
        return it > 0 and it % self.interval == 0


class MaxEpoch(Trigger):
    def __init__(self, max_epoch):
        self.max_epoch = int(max_epoch)

    def __call__(self, state):
        return state["epoch"] > self.max_epoch


class MaxIteration(Trigger):
    iteration_based = True

    def __init__(self, max_iter):
        self.max_iter = int(max_iter)

    def __call__(self, state):
        return state["neval"] > self.max_iter


class MaxScore(Trigger):
    def __init__(self, max_score):
        self.max_score = float(max_score)

    def __call__(self, state):
        s = state.get("score")
        return s is not None and s > self.max_score


class MinLoss(Trigger):
    iteration_based = True

    def __init__(self, min_loss):
        self.min_loss = float(min_loss)

    def __call__(self, state):
        l = state.get("Loss")
        return l is not None and l == l and l < self.min_loss


class And(Trigger):
    def __init__(self, first, *others):
        self.ts = (first,) + others
        self.iteration_based = all(t.iteration_based for t in self.ts)

    def __call__(self, state):
        return all(t(state) for t in self.ts)


class Or(Trigger):
    def __init__(self, first, *others):
        self.ts = (first,) + others
        self.iteration_based = any(t.iteration_based for t in self.ts)

    def __call__(self, state):
        return any(t(state) for t in self.ts)


# reference aliases (ZooTrigger names)
ZooTrigger = Trigger
