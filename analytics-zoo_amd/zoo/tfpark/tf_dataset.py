"""TFDataset (Py/tfpark/tf_dataset.py:TFDataset.from_*) -> FeatureSet."""
import numpy as np

from zoo.feature.common import FeatureSet


class TFDataset:
    def __init__(self, train, val=None, batch_size=32, batch_per_thread=-1, hard_code_batch_size=False):
        self.train, self.val = train, val
        self.batch_size, self.batch_per_thread = batch_size, batch_per_thread

    def get_training_data(self):
        return self.train

    def get_validation_data(self):
        return self.val

    def get_prediction_data(self):
        return self.train

    def get_evaluation_data(self):
        return self.val or self.train

    def get_num_partitions(self):
        from zoo.common.nncontext import get_nncontext
        return get_nncontext().world_size

    @staticmethod
    def _bs(batch_size, batch_per_thread):
        return batch_size if batch_size and batch_size > 0 else (batch_per_thread if batch_per_thread > 0 else 32)

    @staticmethod
    def from_ndarrays(tensors, batch_size=-1, batch_per_thread=-1, hard_code_batch_size=False, val_tensors=None,
                      memory_type="DRAM"):
        bs = TFDataset._bs(batch_size, batch_per_thread)
        x, y = (tensors[0], tensors[1]) if isinstance(tensors, tuple) and len(tensors) == 2 else (tensors, None)
        train = FeatureSet.from_ndarrays(x, y, bs, shuffle=batch_size > 0)
        val = None
        if val_tensors is not None:
            vx, vy = val_tensors if isinstance(val_tensors, tuple) else (val_tensors, None)
            val = FeatureSet.from_ndarrays(vx, vy, bs, shuffle=False)
        return TFDataset(train, val, batch_size, batch_per_thread)

    @staticmethod
    def from_feature_set(dataset, features=None, labels=None, batch_size=-1, batch_per_thread=-1,
                         hard_code_batch_size=False, validation_dataset=None):
        return TFDataset(dataset, validation_dataset, batch_size, batch_per_thread)

    @staticmethod
    def from_image_set(image_set, image=None, label=None, batch_size=-1, batch_per_thread=-1,
                       hard_code_batch_size=False, validation_image_set=None):
        bs = TFDataset._bs(batch_size, batch_per_thread)
        val = validation_image_set.to_featureset(bs, shuffle=False) if validation_image_set is not None else None
        return TFDataset(image_set.to_featureset(bs, shuffle=batch_size > 0), val, batch_size, batch_per_thread)

    @staticmethod
    def from_text_set(text_set, text=None, label=None, batch_size=-1, batch_per_thread=-1,
                      hard_code_batch_size=False, validation_text_set=None):
        bs = TFDataset._bs(batch_size, batch_per_thread)
        val = validation_text_set.to_featureset(bs, shuffle=False) if validation_text_set is not None else None
        return TFDataset(text_set.to_featureset(bs, shuffle=batch_size > 0), val, batch_size, batch_per_thread)

    @staticmethod
    def from_dataframe(df, feature_cols, labels_cols=None, batch_size=-1, batch_per_thread=-1,
                       hard_code_batch_size=False, validation_df=None):
        bs = TFDataset._bs(batch_size, batch_per_thread)

        def arrays(d):
            x = np.stack([np.concatenate([np.asarray(r[c], np.float32).reshape(-1) for c in feature_cols])
                          for _, r in d.iterrows()])
            y = None
            if labels_cols:
                y = np.stack([np.concatenate([np.asarray(r[c], np.float32).reshape(-1) for c in labels_cols])
                              for _, r in d.iterrows()])
                y = y[:, 0] if y.shape[1] == 1 else y
            return x, y
        x, y = arrays(df)
        val = FeatureSet.from_ndarrays(*arrays(validation_df), bs, shuffle=False) if validation_df is not None \
            else None
        return TFDataset(FeatureSet.from_ndarrays(x, y, bs, shuffle=batch_size > 0), val, batch_size,
                         batch_per_thread)

    @staticmethod
    def from_tf_data_dataset(*a, **k):
        raise NotImplementedError("tf.data needs TensorFlow; build the pipeline with FeatureSet / DataLoader")

    @staticmethod
    def from_tfrecord_file(*a, **k):
        raise NotImplementedError("TFRecord decoding of tf.Example needs TensorFlow protos; use FeatureSet")

    from_rdd = from_feature_set
