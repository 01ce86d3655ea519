"""TF1-style parameter-server entry point for the TensorHive ClusterSpec example.

TensorHive's `tf1` template passes ``--ps_hosts``, ``--worker_hosts``, ``--job_name`` and
``--task_index`` (ports assigned from 2222 upward) and sets ``HIP_VISIBLE_DEVICES`` per worker
(empty for parameter servers).  This script parses and checks them the way a TF1 program builds
its ``tf.train.ClusterSpec``; with TensorFlow installed it starts the ``tf.distribute.Server``.
"""
import argparse
import os
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ps_hosts", required=True)
    ap.add_argument("--worker_hosts", required=True)
    ap.add_argument("--job_name", choices=["ps", "worker"], required=True)
    ap.add_argument("--task_index", type=int, required=True)
    a = ap.parse_args()
    cluster = {"ps": [h for h in a.ps_hosts.split(",") if h], "worker": [h for h in a.worker_hosts.split(",") if h]}
    me = cluster[a.job_name][a.task_index]
    print(f"[tf1] job={a.job_name}:{a.task_index} address={me} ps={len(cluster['ps'])} "
          f"workers={len(cluster['worker'])} gpus={os.environ.get('HIP_VISIBLE_DEVICES', '')!r}", flush=True)
    try:
        import tensorflow as tf  # noqa: F401
    except ImportError:
        print("[tf1] tensorflow not installed: cluster view only", flush=True)
        return 0
    server = tf.distribute.Server(tf.train.ClusterSpec(cluster), job_name=a.job_name, task_index=a.task_index)
    if a.job_name == "ps":
        server.join()
    return 0


if __name__ == "__main__":
    sys.exit(main())
