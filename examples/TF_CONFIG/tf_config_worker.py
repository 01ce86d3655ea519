"""TF2 multi-worker entry point for the TensorHive TF_CONFIG example.

TensorHive's `tf2` template gives every task a persisted ``TF_CONFIG`` (cluster + this task's type
and index) and its GPU in ``HIP_VISIBLE_DEVICES``.  With TensorFlow-ROCm installed this script
builds ``tf.distribute.MultiWorkerMirroredStrategy`` from it and trains a small Keras model on
synthetic data; without TensorFlow (as in this repository's test image) it validates and prints
the cluster view it was given, which is what the launch tests check.
"""
import json
import os
import sys


def main() -> int:
    raw = os.environ.get("TF_CONFIG")
    if not raw:
        print("[tf2] TF_CONFIG is not set", file=sys.stderr)
        return 2
    cfg = json.loads(raw)
    cluster, task = cfg["cluster"], cfg["task"]
    me = cluster[task["type"]][task["index"]]
    workers = sum(len(v) for k, v in cluster.items() if k in ("chief", "worker"))
    print(f"[tf2] task={task['type']}:{task['index']} address={me} workers={workers} "
          f"gpus={os.environ.get('HIP_VISIBLE_DEVICES', '')}", flush=True)
    try:
        import tensorflow as tf  # noqa: F401  (TensorFlow-ROCm, optional)
    except ImportError:
        print("[tf2] tensorflow not installed: cluster view only", flush=True)
        return 0
    strategy = tf.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        model = tf.keras.Sequential([tf.keras.layers.Dense(512, activation="gelu"), tf.keras.layers.Dense(10)])
        model.compile(optimizer="adam", loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True))
    x = tf.random.normal((4096, 256))
    y = tf.random.uniform((4096,), maxval=10, dtype=tf.int32)
    model.fit(x, y, epochs=2, batch_size=128 * strategy.num_replicas_in_sync, verbose=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
