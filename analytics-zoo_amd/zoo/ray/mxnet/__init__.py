"""Synchronous distributed trainer over RayContext actors
(Py/ray/mxnet/mxnet_trainer.py:26-145, mxnet_runner.py:28-215, utils.py:28-45).

The reference runs MXNet workers + parameter servers (``dist_sync`` kvstore
over ps-lite) as Ray actors. Here the same entry points drive the framework's
own engine: every worker actor joins one torch.distributed group (RCCL on
GPUs, gloo on CPU; SURVEY.md §2.14 P7 "replaced by P1"), builds its model /
loss / data with the user's creator functions and trains with the bucketed
all-reduce of zoo.parallel.ddp. ``num_servers`` is accepted for API parity;
no server processes are needed because the reduction is collective.

Creators follow the reference signatures:
  data_creator(config, kv)  -> train data or (train, val); ``kv.rank`` and
                               ``kv.num_workers`` shard the data
  model_creator(config)     -> torch.nn.Module (any zoo Keras model qualifies)
  loss_creator(config)      -> criterion(output, target) or a loss name
  metrics_creator(config)   -> metric name(s) / ValidationMethod(s)
"""
import logging
import os
import socket
import time

from zoo.ray.raycontext import RayContext, get, remote

log = logging.getLogger("zoo.ray")


def find_free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def create_trainer_config(batch_size=32, optimizer="sgd", optimizer_params=None, log_interval=10, seed=None,
                          extra_config=None):
    config = {"batch_size": batch_size, "optimizer": optimizer,
              "optimizer_params": optimizer_params or {"learning_rate": 0.01}, "log_interval": log_interval}
    if seed:
        config["seed"] = seed
    if extra_config:
        assert isinstance(extra_config, dict), "extra_config must be a dict"
        config.update(extra_config)
    return config


class _KV:
    """What data_creator receives in place of the MXNet kvstore handle."""

    def __init__(self, rank, num_workers):
        self.rank, self.num_workers = rank, num_workers
        self.type = "dist_sync"


def _make_optim(name, params):
    from zoo.pipeline.api.keras import optimizers as O
    if isinstance(name, O.OptimMethod):
        return name
    p = dict(params or {})
    lr = p.pop("learning_rate", p.pop("lr", 0.01))
    wd = p.pop("wd", p.pop("weight_decay", 0.0))
    n = str(name).lower()
    if n == "sgd":
        return O.SGD(learningrate=lr, weightdecay=wd, momentum=p.pop("momentum", 0.0))
    if n == "adam":
        return O.Adam(lr=lr, beta_1=p.pop("beta1", 0.9), beta_2=p.pop("beta2", 0.999),
                      epsilon=p.pop("epsilon", 1e-8))
    return O.to_optim_method(n)


class TrainingRunner:
    """One worker actor (MXNetRunner's role)."""

    def get_node_ip(self):
        return "127.0.0.1"

    def find_free_port(self):
        return find_free_port()

    def setup_distributed(self, env, config, data_creator, model_creator, loss_creator=None, metrics_creator=None):
        import torch
        for k in ("batch_size", "optimizer", "optimizer_params", "log_interval"):
            assert k in config, k + " must be specified in config"
        os.environ.update({k: str(v) for k, v in env.items()})
        from zoo.common.nncontext import init_nncontext
        from zoo.pipeline.api.keras.metrics import to_metrics
        from zoo.pipeline.api.keras.objectives import to_criterion
        from zoo.pipeline.engine import TrainingEngine
        if "seed" in config:
            torch.manual_seed(int(config["seed"]))  # identical init on every worker
        self.ctx = init_nncontext(backend=config.get("backend", ""), seed=int(config.get("seed", 1)))
        self.config = config
        kv = _KV(self.ctx.rank, self.ctx.world_size)
        data = data_creator(config, kv)
        if isinstance(data, tuple):
            assert len(data) in (1, 2), "data_creator returns train_data or (train_data, val_data)"
            self.train_data, self.val_data = (data[0], None) if len(data) == 1 else data
        else:
            self.train_data, self.val_data = data, None
        model = model_creator(config)
        assert loss_creator is not None, "Loss not defined, please specify loss_creator"
        loss = loss_creator(config)
        self.criterion = to_criterion(loss) if isinstance(loss, str) else loss
        self.metrics = None
        if self.val_data is not None:
            assert metrics_creator, "Metrics not defined for validation, please specify metrics_creator"
            self.metrics = to_metrics(metrics_creator(config), self.criterion)
        self.engine = TrainingEngine(model, self.criterion, _make_optim(config["optimizer"],
                                                                         config["optimizer_params"]))
        return True

    def train(self, nb_epoch=1):
        stats = {}
        eng, cfg = self.engine, self.config
        t0 = time.time()
        for epoch in range(nb_epoch):
            n, losses, te = 0, [], time.time()
            for i, batch in enumerate(self.train_data):
                x, y = batch[0], batch[1]
                loss = eng.train_step(x, y)
                n += len(y)
                if (i + 1) % int(cfg["log_interval"]) == 0:
                    losses.append(float(loss))
                    log.info("Epoch[%d] Batch[%d] Speed: %.1f samples/sec loss=%.4f", epoch, i,
                             n / max(time.time() - te, 1e-9), losses[-1])
            losses.append(float(loss))
            stats["epoch"] = epoch
            stats["loss"] = losses[-1]
            stats["epoch_time"] = time.time() - te
            stats["samples_per_sec"] = n / max(stats["epoch_time"], 1e-9)
            if self.metrics:
                for name, res in eng.evaluate(self.val_data, self.metrics):
                    stats[name] = float(res[0]) if isinstance(res, (tuple, list)) else float(res)
        stats["time"] = time.time() - t0
        return stats

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.engine.model.state_dict().items()}

    def shutdown(self):
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
        return True


class MXNetTrainer:
    def __init__(self, config, data_creator, model_creator, loss_creator=None, metrics_creator=None,
                 num_workers=1, num_servers=None, runner_cores=None):
        self.config = config
        self.num_workers = int(num_workers)
        self.num_servers = num_servers if num_servers else self.num_workers  # API parity only
        RayContext.get(initialize=True)
        Worker = remote(num_cpus=runner_cores)(TrainingRunner)
        self.runners = [Worker.remote() for _ in range(self.num_workers)]
        port = find_free_port()
        envs = [{"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port, "RANK": i, "WORLD_SIZE": self.num_workers,
                 "LOCAL_RANK": i} for i in range(self.num_workers)]
        get([r.setup_distributed.remote(envs[i], config, data_creator, model_creator, loss_creator,
                                        metrics_creator) for i, r in enumerate(self.runners)])

    def train(self, nb_epoch=1):
        return get([w.train.remote(nb_epoch) for w in self.runners])

    def get_weights(self):
        return get(self.runners[0].get_weights.remote())

    def shutdown(self):
        get([w.shutdown.remote() for w in self.runners])
        for w in self.runners:
            RayContext.kill(w)
        self.runners = []


DistributedTrainer = MXNetTrainer
