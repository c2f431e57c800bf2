"""oryx-run CLI (deploy/bin/oryx-run.sh equivalent): topic setup, input, tail, config dump."""

import io
import os
import subprocess
import sys

from oryx_amd import cli
from oryx_amd.transport import log as tlog

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _conf_file(tmp_path):
    p = tmp_path / "app.conf"
    p.write_text('oryx {\n  id = "cli-test"\n  input-topic.broker = "log:%s/log"\n'
                 '  update-topic.broker = "log:%s/log"\n  serving.api.password = "secret"\n}\n'
                 % (tmp_path, tmp_path))
    return str(p)


def test_log_setup_input_tail(tmp_path):
    conf = cli._load_config(_conf_file(tmp_path), set_env=False)
    out = io.StringIO()
    cli.cmd_log_setup(conf, out)
    assert "Created topic OryxInput" in out.getvalue()
    t = tlog.Topic(str(tmp_path / "log"), "OryxInput")
    assert t.partitions == 4
    assert tlog.Topic(str(tmp_path / "log"), "OryxUpdate").partitions == 1
    data = tmp_path / "in.csv"
    data.write_text("a,b,1\nc,d,2\n\ne,f,3\n")
    assert cli.cmd_log_input(conf, str(data), io.StringIO()) == 3
    assert sum(t.end_offsets()) == 3
    out = io.StringIO()
    cli.cmd_log_setup(conf, out)
    assert "Existing topic OryxInput" in out.getvalue()


def test_config_props_redacts(tmp_path):
    conf = cli._load_config(_conf_file(tmp_path), set_env=False)
    out = io.StringIO()
    cli.cmd_config_props(conf, out)
    text = out.getvalue()
    assert "oryx.id=cli-test" in text
    assert "oryx.batch.streaming.generation-interval-sec=" in text


def test_wrapper_script_help():
    r = subprocess.run([os.path.join(ROOT, "bin", "oryx-run"), "--help"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "log-setup" in r.stdout
