"""Drop-in for lib/utils.py host helpers (init_network_weights :69-73,
update_learning_rate :75-79, make_file :81-84, append_to_line :58-67)."""
import os

import torch.nn as nn


def init_network_weights(net, std=0.1):
    """N(0, std) weights, zero biases for every nn.Linear in ``net``."""
    for m in net.modules():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0, std=std)
            nn.init.constant_(m.bias, val=0)


def update_learning_rate(optimizer, decay_rate=0.999, lowest=1e-3):
    for group in optimizer.param_groups:
        group["lr"] = max(group["lr"] * decay_rate, lowest)


def make_file(prefix):
    folder = os.path.dirname(prefix)
    if folder and not os.path.exists(folder):
        os.makedirs(folder)


def append_to_line(file_path, line_prefix, append="finished"):
    from filelock import FileLock
    with FileLock(file_path + ".lock"):
        with open(file_path) as f:
            rows = f.readlines()
        with open(file_path, "w") as f:
            for row in rows:
                f.write(row.rstrip("\n") + " " + append + "\n" if row.startswith(line_prefix) else row)
