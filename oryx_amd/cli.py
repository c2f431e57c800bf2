"""``oryx-run``: launch a layer or administer the update/input logs.

Equivalent of ``deploy/bin/oryx-run.sh`` (``:18-38`` usage, ``:117-299`` layers, ``:301-365``
topic commands) and the per-layer ``Main`` classes (``deploy/oryx-{batch,speed,serving}/.../
Main.java:31-37``) plus ``ConfigToProperties`` (``[common]/settings/ConfigToProperties.java:
33-58``)::

    python -m oryx_amd.cli batch   --conf app.conf [--gpus N]
    python -m oryx_amd.cli speed   --conf app.conf
    python -m oryx_amd.cli serving --conf app.conf
    python -m oryx_amd.cli log-setup --conf app.conf        (alias: kafka-setup)
    python -m oryx_amd.cli log-tail  --conf app.conf        (alias: kafka-tail)
    python -m oryx_amd.cli log-input --conf app.conf --input-file data.csv  (alias: kafka-input)
    python -m oryx_amd.cli config-props --conf app.conf     (key=value dump)

``batch --gpus N`` (N > 1) re-launches itself under ``torch.distributed.run`` with one rank per
GPU (127.0.0.1 rendezvous); rank 0 drives the layer and every rank joins the collective
training calls.  Layers run until interrupted (Ctrl-C / SIGTERM closes them in LIFO order).
"""

from __future__ import annotations

import argparse
import logging
import os
import signal
import subprocess
import sys
import threading
import time
from typing import List, Optional

__all__ = ["main"]

log = logging.getLogger("oryx_amd.cli")

_ALIASES = {"kafka-setup": "log-setup", "kafka-tail": "log-tail", "kafka-input": "log-input"}


def _load_config(path: Optional[str], set_env: bool = True):
    from .utils import config as cfg
    if path:
        if set_env:     # so that code calling cfg.get_default() in this process sees it too
            os.environ["ORYX_CONFIG_FILE"] = os.path.abspath(path)
        return cfg.load_file(path)
    return cfg.get_default()


def _wait_forever(layer) -> None:
    stop = threading.Event()

    def handler(signum, frame):
        stop.set()

    signal.signal(signal.SIGINT, handler)
    signal.signal(signal.SIGTERM, handler)
    try:
        while not stop.is_set():
            stop.wait(1.0)
    finally:
        layer.close()


def _topics(config):
    from .transport import log as tlog
    in_root = tlog.log_root_for(config.get_string("oryx.input-topic.broker"), config)
    up_root = tlog.log_root_for(config.get_string("oryx.update-topic.broker"), config)
    return (in_root, config.get_string("oryx.input-topic.message.topic"),
            up_root, config.get_string("oryx.update-topic.message.topic"))


def cmd_log_setup(config, out=sys.stdout) -> None:
    from .transport import log as tlog
    in_root, in_topic, up_root, up_topic = _topics(config)
    max_msg = config.get_int("oryx.update-topic.message.max-size")
    for root, topic, parts in ((in_root, in_topic, config.get_int("oryx.input-topic.partitions")),
                               (up_root, up_topic, config.get_int("oryx.update-topic.partitions"))):
        existed = tlog.topic_exists(root, topic)
        tlog.maybe_create_topic(root, topic, parts, max_message=max_msg)
        t = tlog.Topic(root, topic)
        print("%s topic %s in %s: %d partitions, end offsets %s" % (
            "Existing" if existed else "Created", topic, root, t.partitions, t.end_offsets()),
            file=out)
        t.close()


def cmd_log_tail(config, out=sys.stdout, max_seconds: Optional[float] = None) -> None:
    from .transport import log as tlog
    in_root, in_topic, up_root, up_topic = _topics(config)
    consumers = []
    for root, topic in ((in_root, in_topic), (up_root, up_topic)):
        if tlog.topic_exists(root, topic):
            consumers.append((topic, tlog.TopicConsumer(tlog.Topic(root, topic), "latest")))
    t0 = time.time()
    try:
        while max_seconds is None or time.time() - t0 < max_seconds:
            got = False
            for name, c in consumers:
                for _, _, _, k, m in c.poll(1024, 100):
                    got = True
                    print("%s\t%s\t%s" % (name, k, m if len(m) < 2000 else m[:2000] + "..."),
                          file=out, flush=True)
            if not got:
                time.sleep(0.1)
    except KeyboardInterrupt:
        pass
    finally:
        for _, c in consumers:
            c.close()


def cmd_log_input(config, input_file: str, out=sys.stdout) -> int:
    from .transport.producer import LogTopicProducer
    if not os.path.isfile(input_file):
        raise SystemExit("Input file %s does not exist" % input_file)
    in_root, in_topic, _, _ = _topics(config)
    prod = LogTopicProducer(config.get_string("oryx.input-topic.broker"), in_topic, config,
                            async_=False,
                            create_partitions=config.get_int("oryx.input-topic.partitions"))
    n = 0
    with open(input_file, "r", encoding="utf-8") as f:
        batch = []
        for line in f:
            line = line.rstrip("\n")
            if line:
                batch.append((None, line))
            if len(batch) >= 1000:
                prod.send_many(batch)
                n += len(batch)
                batch = []
        if batch:
            prod.send_many(batch)
            n += len(batch)
    prod.close()
    print("Sent %d lines to %s" % (n, in_topic), file=out)
    return n


def cmd_config_props(config, out=sys.stdout) -> None:
    from .utils import config as cfg
    print(cfg.to_properties(config), file=out)


def _relaunch_distributed(argv: List[str], gpus: int, max_restarts: int = 0,
                          min_gpus: int = 1) -> int:
    # a rank that fails (or is ended by the watchdog) makes the agent restart the whole group
    # up to max_restarts times; the ALS trainer then resumes from its factor checkpoint.  A
    # rank that loses its GPU ends the group instead, and the supervisor relaunches it on a
    # smaller world of the healthy GPUs (parallel/elastic.py)
    from .parallel import elastic

    def build(world: int) -> List[str]:
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                "--nproc-per-node=%d" % world, "--max-restarts=%d" % max_restarts,
                "--master-addr=127.0.0.1",
                "--master-port=%s" % os.environ.get("ORYX_MASTER_PORT", "29551"),
                "-m", "oryx_amd.cli"] + _with_gpus(argv, world)
    env = dict(os.environ, ORYX_DISTRIBUTED_CHILD="1")
    return elastic.supervise(build, gpus, min_world=min_gpus, env=env)


def _with_gpus(argv: List[str], world: int) -> List[str]:
    """``argv`` with its ``--gpus`` value replaced by ``world``."""
    out, skip = [], False
    for j, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a == "--gpus":
            out += ["--gpus", str(world)]
            skip = True
        elif a.startswith("--gpus="):
            out.append("--gpus=%d" % world)
        else:
            out.append(a)
    return out


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="oryx-run", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("command", choices=["batch", "speed", "serving", "log-setup", "log-tail",
                                        "log-input", "config-props"] + list(_ALIASES))
    ap.add_argument("--conf", help="HOCON config file (overlaid on the defaults)")
    ap.add_argument("--input-file", help="log-input: file of input lines")
    ap.add_argument("--gpus", type=int, default=1, help="batch: ranks (one per GPU)")
    ap.add_argument("--log-level", default=os.environ.get("ORYX_LOG_LEVEL", "INFO"))
    args = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(levelname)-5s %(name)s: %(message)s")
    command = _ALIASES.get(args.command, args.command)
    config = _load_config(args.conf)
    from .utils import config as cfg
    if command == "log-setup":
        cmd_log_setup(config)
        return 0
    if command == "log-tail":
        cmd_log_tail(config)
        return 0
    if command == "log-input":
        if not args.input_file:
            ap.error("--input-file is required")
        cmd_log_input(config, args.input_file)
        return 0
    if command == "config-props":
        cmd_config_props(config)
        return 0
    log.info("Configuration:\n%s", cfg.pretty_print(config))
    if command == "batch":
        if args.gpus > 1 and not os.environ.get("ORYX_DISTRIBUTED_CHILD"):
            return _relaunch_distributed(
                argv, args.gpus, cfg.get_optional_int(config, "oryx.gpu.max-restarts") or 0,
                cfg.get_optional_int(config, "oryx.gpu.elastic.min-gpus") or 1)
        from .layers.batch import BatchLayer
        from .parallel import dist, elastic
        try:
            ctx = dist.init_from_env(device=config.get_string("oryx.gpu.device"))
            layer = BatchLayer(config)
            if ctx.is_main:
                layer.start()
                _wait_forever(layer)
            else:
                layer.run_follower()
        except Exception as e:
            if os.environ.get("ORYX_DISTRIBUTED_CHILD") and elastic.is_device_failure(e):
                elastic.report_device_lost(str(e))
            raise
        return 0
    if command == "speed":
        from .layers.speed import SpeedLayer
        layer = SpeedLayer(config).start()
        _wait_forever(layer)
        return 0
    if command == "serving":
        from .serving.layer import ServingLayer
        layer = ServingLayer(config).start()
        log.info("Serving on port %d", layer.actual_port)
        _wait_forever(layer)
        return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
