"""Packaging surface (reference C10/C11: install scripts, bin entry, version)."""
import importlib
import os
import re
import subprocess
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _console_scripts():
    src = open(os.path.join(ROOT, "setup.py")).read()
    return dict(re.findall(r'"([\w-]+) = ([\w.:]+)"', src))


def test_console_scripts_resolve():
    scripts = _console_scripts()
    assert {"symmetry-cli", "symmetry-dht", "symmetry-server", "symmetry-client"} <= set(scripts)
    for name, target in scripts.items():
        mod, fn = target.split(":")
        assert callable(getattr(importlib.import_module(mod), fn)), name


def test_install_scripts_parse():
    subprocess.run(["bash", "-n", os.path.join(ROOT, "install.sh")], check=True)
    ps1 = open(os.path.join(ROOT, "install.ps1")).read()
    assert "symmetry_amd.cli --init" in ps1


def test_cli_init_writes_install_defaults(tmp_path):
    out = subprocess.run([sys.executable, "-m", "symmetry_amd.cli", "--version"], capture_output=True, text=True,
                         cwd=ROOT, check=True)
    assert out.stdout.strip() == "1.0.0"  # reference src/symmetry.ts:11
    cfg = tmp_path / "symmetry" / "provider.yaml"
    subprocess.run([sys.executable, "-m", "symmetry_amd.cli", "--init", "-c", str(cfg)], cwd=ROOT, check=True,
                   capture_output=True)
    d = yaml.safe_load(cfg.read_text())
    # reference install.sh:37-49 defaults
    assert d["maxConnections"] == 10 and d["dataCollectionEnabled"] is True and d["public"] is True
    assert d["modelName"] == "llama3.1:latest"
    assert d["serverKey"] == "4b4a9cc325d134dee6679e9407420023531fd7e96c563f6c5d00fd5549b77435"
    assert d["path"] == str(cfg.parent)
