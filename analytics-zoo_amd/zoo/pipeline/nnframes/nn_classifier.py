"""NNFrames: DataFrame-level fit/transform (Spark ML Pipelines analogue).

The reference (Zs/pipeline/nnframes/NNEstimator.scala:194-700, NNClassifier.scala:42-306,
Python Py/pipeline/nnframes/nn_classifier.py:29-581) plugs BigDL models into
Spark ML Estimator/Transformer. There is no Spark here: the DataFrame is a
pandas DataFrame (per-rank shard when running one process per GPU), and
``fit`` goes through the same TrainingEngine as every other front end
(bucketed RCCL all-reduce across ranks). The API — setters, the
feature/label Preprocessing, caching level, validation, checkpoint,
summaries, NNModel.transform and the classifier's 1-based argmax /
threshold prediction (NNClassifier.scala:193-200) — follows the reference.
"""
import copy
import json
import os

import numpy as np
import torch

from zoo.common import triggers as T
from zoo.feature.common import (ChainedPreprocessing, FeatureLabelPreprocessing, FeatureSet, MemoryType,
                                Preprocessing, ScalarToTensor, SeqToMultipleTensors, SeqToTensor)


def _to_preprocessing(p, default):
    if p is None or (isinstance(p, list) and not p):
        return default
    if isinstance(p, list):
        if isinstance(p[0], (list, tuple)):
            return SeqToMultipleTensors(p)
        return SeqToTensor(p)
    return p


def _column_tensor(values, prep):
    """Apply a Preprocessing to every row of a column and stack the results.
    SeqToTensor / ScalarToTensor columns are converted in one vectorised step."""
    if type(prep) is SeqToTensor:
        arr = np.stack([np.asarray(v, dtype=np.float32).reshape(-1) for v in values]) if len(values) else \
            np.zeros((0,), np.float32)
        t = torch.from_numpy(arr)
        return t.reshape((len(values),) + tuple(prep.size)) if prep.size else t
    if type(prep) is ScalarToTensor:
        return torch.tensor(np.asarray(values, dtype=np.float32)).reshape(-1, 1)
    rows = [prep(v) for v in values]
    if rows and isinstance(rows[0], (list, tuple)):
        return [torch.stack([torch.as_tensor(r[i]) for r in rows]) for i in range(len(rows[0]))]
    return torch.stack([torch.as_tensor(r) for r in rows])


class _Params:
    def __init__(self):
        self.featuresCol = "features"
        self.labelCol = "label"
        self.predictionCol = "prediction"
        self.batchSize = 32

    def setFeaturesCol(self, v):  # noqa: N802 - reference names
        self.featuresCol = v
        return self

    def getFeaturesCol(self):  # noqa: N802
        return self.featuresCol

    def setLabelCol(self, v):  # noqa: N802
        self.labelCol = v
        return self

    def getLabelCol(self):  # noqa: N802
        return self.labelCol

    def setPredictionCol(self, v):  # noqa: N802
        self.predictionCol = v
        return self

    def getPredictionCol(self):  # noqa: N802
        return self.predictionCol

    def setBatchSize(self, v):  # noqa: N802
        self.batchSize = int(v)
        return self

    def getBatchSize(self):  # noqa: N802
        return self.batchSize


class NNEstimator(_Params):
    def __init__(self, model, criterion, feature_preprocessing=None, label_preprocessing=None):
        super().__init__()
        self.model = model
        self.criterion = criterion
        self.feature_preprocessing = _to_preprocessing(feature_preprocessing, SeqToTensor())
        self.label_preprocessing = _to_preprocessing(label_preprocessing, SeqToTensor())
        self.samplePreprocessing = FeatureLabelPreprocessing(self.feature_preprocessing, self.label_preprocessing)
        self.maxEpoch = 50
        self.learningRate = 1e-3
        self.learningRateDecay = 0.0
        self.optimMethod = None
        self.endWhen = None
        self.cachingSample = True
        self.dataCacheLevel = ("DRAM", None)
        self.train_summary = None
        self.validation_summary = None
        self.validation_config = None
        self.checkpoint_config = None
        self._clip = None
        self.engine = None
        self.localPartition = False

    # -- setters mirroring nn_classifier.py:224-437 --------------------------
    def setSamplePreprocessing(self, val):  # noqa: N802
        self.samplePreprocessing = val
        return self

    def getSamplePreprocessing(self):  # noqa: N802
        return self.samplePreprocessing

    def setOptimMethod(self, val):  # noqa: N802
        self.optimMethod = val
        return self

    def getOptimMethod(self):  # noqa: N802
        return self.optimMethod

    def setMaxEpoch(self, val):  # noqa: N802
        self.maxEpoch = int(val)
        return self

    def getMaxEpoch(self):  # noqa: N802
        return self.maxEpoch

    def setEndWhen(self, trigger):  # noqa: N802
        self.endWhen = trigger
        return self

    def getEndWhen(self):  # noqa: N802
        return self.endWhen

    def setDataCacheLevel(self, level, numSlice=None):  # noqa: N802
        level = level.upper()
        if level not in ("DRAM", "DIRECT", "PMEM", "DEVICE", "DISK_AND_DRAM"):
            raise ValueError("unknown cache level %s" % level)
        if level == "DISK_AND_DRAM" and not numSlice:
            raise ValueError("DISK_AND_DRAM needs numSlice")
        self.dataCacheLevel = (level, numSlice)
        return self

    def getDataCacheLevel(self):  # noqa: N802
        return self.dataCacheLevel[0]

    def setLocalPartition(self, val=True):  # noqa: N802
        """With one process per GPU: the DataFrame given to fit() is THIS rank's partition (as a
        Spark DataFrame partition lives on its executor), not the whole dataset every rank
        shards. All ranks must pass partitions of equal size; the batch size stays global."""
        self.localPartition = bool(val)
        return self

    def isLocalPartition(self):  # noqa: N802
        return self.localPartition

    def setLearningRate(self, val):  # noqa: N802
        self.learningRate = float(val)
        return self

    def getLearningRate(self):  # noqa: N802
        return self.learningRate

    def setLearningRateDecay(self, val):  # noqa: N802
        self.learningRateDecay = float(val)
        return self

    def getLearningRateDecay(self):  # noqa: N802
        return self.learningRateDecay

    def setCachingSample(self, val):  # noqa: N802
        self.cachingSample = bool(val)
        return self

    def isCachingSample(self):  # noqa: N802
        return self.cachingSample

    def setTrainSummary(self, val):  # noqa: N802
        self.train_summary = val
        return self

    def getTrainSummary(self):  # noqa: N802
        return self.train_summary

    def setValidationSummary(self, val):  # noqa: N802
        self.validation_summary = val
        return self

    def getValidationSummary(self):  # noqa: N802
        return self.validation_summary

    def setValidation(self, trigger, val_df, val_method, batch_size):  # noqa: N802
        self.validation_config = (trigger, val_df, val_method, int(batch_size))
        return self

    def getValidation(self):  # noqa: N802
        return self.validation_config

    def clearGradientClipping(self):  # noqa: N802
        self._clip = None
        return self

    def setConstantGradientClipping(self, min, max):  # noqa: N802,A002
        from zoo.parallel.ddp import constant_clip
        self._clip = constant_clip(float(min), float(max))
        return self

    def setGradientClippingByL2Norm(self, clip_norm):  # noqa: N802
        from zoo.parallel.ddp import global_norm_clip
        self._clip = global_norm_clip(float(clip_norm))
        return self

    def setCheckpoint(self, path, trigger, isOverWrite=True):  # noqa: N802,N803
        self.checkpoint_config = (path, trigger, isOverWrite)
        return self

    def getCheckpoint(self):  # noqa: N802
        return self.checkpoint_config

    # -- data ----------------------------------------------------------------
    def _featureset(self, df, batch_size, shuffle):
        feats = _column_tensor(list(df[self.featuresCol].values), self.feature_preprocessing)
        labels = _column_tensor(list(df[self.labelCol].values), self.label_preprocessing)
        level, nslice = self.dataCacheLevel
        mt = {"DRAM": MemoryType.DRAM, "DIRECT": MemoryType.DIRECT, "PMEM": MemoryType.PMEM,
              "DEVICE": MemoryType.DEVICE}.get(level)
        if level == "DISK_AND_DRAM":
            mt = MemoryType.DISK_AND_DRAM(nslice)
        from zoo.feature.common import DataStrategy
        strategy = DataStrategy.LOCAL if self.localPartition else DataStrategy.PARTITIONED
        return FeatureSet.from_ndarrays(feats, labels, batch_size, shuffle=shuffle, memory_type=mt,
                                        data_strategy=strategy)

    def _label_for_criterion(self, y):
        return y

    def _optim(self):
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        if self.optimMethod is not None:
            return to_optim_method(self.optimMethod)
        return _default_sgd(self.learningRate, self.learningRateDecay)  # NNEstimator.scala default: SGD

    def fit(self, df):
        """NNEstimator.internalFit (NNEstimator.scala:414-470)."""
        from zoo.pipeline.api.keras.objectives import to_criterion
        from zoo.pipeline.engine import TrainingEngine
        crit = to_criterion(self.criterion)
        squeeze = self._squeeze_label()
        loss_fn = (lambda o, t: crit(o, t.reshape(-1))) if squeeze else crit
        eng = TrainingEngine(self.model, loss_fn, self._optim(), clip=self._clip)
        eng.train_summary, eng.val_summary = self.train_summary, self.validation_summary
        if self.checkpoint_config is not None:
            path, trig, ow = self.checkpoint_config
            eng.set_checkpoint(path, trig, ow)
        data = self._featureset(df, self.batchSize, True)
        val = val_methods = val_trigger = None
        if self.validation_config is not None:
            val_trigger, vdf, vm, vbs = self.validation_config
            from zoo.pipeline.api.keras.metrics import to_metrics
            val = self._featureset(vdf, vbs, False)
            val_methods = to_metrics(vm, crit)
        end = self.endWhen or T.MaxEpoch(self.maxEpoch)
        # per-iteration callbacks (engine, state): monitoring hooks, e.g. bench.py --input featureset
        eng.fit(data, end_trigger=end, validation=val, val_methods=val_methods, val_trigger=val_trigger,
                callbacks=getattr(self, "_train_callbacks", ()))
        self.engine = eng
        return self._create_model()

    def _squeeze_label(self):
        return False

    def _create_model(self):
        m = NNModel(self.model, self.feature_preprocessing)
        m.setFeaturesCol(self.featuresCol).setPredictionCol(self.predictionCol).setBatchSize(self.batchSize)
        return m


def _default_sgd(lr, decay):
    from zoo.pipeline.api.keras.optimizers import SGD
    return SGD(learningrate=lr, learningrate_decay=decay)


class NNModel(_Params):
    """Transformer: appends the model's prediction column (NNEstimator.scala:600-760)."""

    def __init__(self, model, feature_preprocessing=None):
        super().__init__()
        self.model = model
        self.feature_preprocessing = _to_preprocessing(feature_preprocessing, SeqToTensor())

    def setSamplePreprocessing(self, val):  # noqa: N802
        self.feature_preprocessing = val
        return self

    @torch.no_grad()
    def _predict(self, df):
        from zoo.common.nncontext import get_nncontext
        dev = get_nncontext().device
        self.model.to(dev)
        was = self.model.training
        self.model.eval()
        x = _column_tensor(list(df[self.featuresCol].values), self.feature_preprocessing)
        n = (x[0] if isinstance(x, list) else x).shape[0]
        outs = []
        for s in range(0, n, self.batchSize):
            chunk = [t[s:s + self.batchSize].to(dev) for t in x] if isinstance(x, list) else \
                x[s:s + self.batchSize].to(dev)
            o = self.model(chunk)
            outs.append(o.float().cpu())
        self.model.train(was)
        return torch.cat(outs).numpy() if outs else np.zeros((0,))

    def _to_prediction(self, out):
        return [row.reshape(-1).astype(np.float64).tolist() for row in out]

    def transform(self, df):
        out = self._predict(df)
        res = df.copy()
        res[self.predictionCol] = self._to_prediction(out)
        return res

    # -- persistence -------------------------------------------------------------
    def save(self, path):
        from zoo.pipeline.api.keras.serialization import save_model
        os.makedirs(path, exist_ok=True)
        save_model(self.model, os.path.join(path, "model.zoo"), over_write=True)
        meta = {"class": type(self).__name__, "featuresCol": self.featuresCol, "predictionCol": self.predictionCol,
                "batchSize": self.batchSize, "threshold": getattr(self, "threshold", None),
                "feature_size": getattr(self.feature_preprocessing, "size", None)}
        with open(os.path.join(path, "metadata.json"), "w") as f:
            json.dump(meta, f)
        return self

    @classmethod
    def load(cls, path):
        from zoo.pipeline.api.keras.serialization import load_model
        with open(os.path.join(path, "metadata.json")) as f:
            meta = json.load(f)
        model = load_model(os.path.join(path, "model.zoo"))
        klass = {"NNModel": NNModel, "NNClassifierModel": NNClassifierModel}.get(meta["class"], cls)
        m = klass(model, SeqToTensor(meta.get("feature_size")))
        m.setFeaturesCol(meta["featuresCol"]).setPredictionCol(meta["predictionCol"]).setBatchSize(meta["batchSize"])
        if meta.get("threshold") is not None and hasattr(m, "setThreshold"):
            m.setThreshold(meta["threshold"])
        return m


class NNClassifier(NNEstimator):
    """Label column holds 1-based class ids (BigDL convention); the fitted
    model predicts 1-based class ids, or 0/1 by threshold for one output."""

    def __init__(self, model, criterion, feature_preprocessing=None, zero_based_label=False):
        super().__init__(model, criterion, feature_preprocessing, ScalarToTensor())
        self.zero_based_label = zero_based_label

    def _squeeze_label(self):
        return True

    def fit(self, df):
        from zoo.pipeline.api.keras.objectives import ClassNLLCriterion, to_criterion
        crit = to_criterion(self.criterion)
        if isinstance(crit, ClassNLLCriterion) and not self.zero_based_label and crit.zero_based_label:
            crit = copy.copy(crit)
            crit.zero_based_label = False
        self.criterion = crit
        return super().fit(df)

    def _create_model(self):
        m = NNClassifierModel(self.model, self.feature_preprocessing)
        m.setFeaturesCol(self.featuresCol).setPredictionCol(self.predictionCol).setBatchSize(self.batchSize)
        m.zero_based_label = self.zero_based_label
        return m


class NNClassifierModel(NNModel):
    def __init__(self, model, feature_preprocessing=None):
        super().__init__(model, feature_preprocessing)
        self.threshold = 0.5
        self.zero_based_label = False

    def setThreshold(self, v):  # noqa: N802
        self.threshold = float(v)
        return self

    def getThreshold(self):  # noqa: N802
        return self.threshold

    def _to_prediction(self, out):
        out = out.reshape(out.shape[0], -1)
        if out.shape[1] == 1:
            return (out[:, 0] > self.threshold).astype(np.float64).tolist()
        cls = out.argmax(1) + (0 if self.zero_based_label else 1)
        return cls.astype(np.float64).tolist()


class Pipeline:
    """Minimal Spark-ML-style pipeline: fit each estimator stage in turn."""

    def __init__(self, stages):
        self.stages = stages

    def fit(self, df):
        fitted = []
        for st in self.stages:
            if hasattr(st, "fit"):
                st = st.fit(df)
            df = st.transform(df)
            fitted.append(st)
        return PipelineModel(fitted)


class PipelineModel:
    def __init__(self, stages):
        self.stages = stages

    def transform(self, df):
        for st in self.stages:
            df = st.transform(df)
        return df


__all__ = ["NNEstimator", "NNModel", "NNClassifier", "NNClassifierModel", "Pipeline", "PipelineModel",
           "Preprocessing", "ChainedPreprocessing"]
