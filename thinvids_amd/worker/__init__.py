"""Worker side of the cluster (reference worker/tasks.py): helper layer, data-plane HTTP
server, segment encoder and the transcode/split/encode/stitch/stamp tasks."""
