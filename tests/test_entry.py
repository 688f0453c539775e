"""The driver entry points run on CPU too (the service never needs the GPU)."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def load_entry():
    spec = importlib.util.spec_from_file_location("graft_entry", ROOT / "__graft_entry__.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_smoke_runs(hola_bin, capsys):
    load_entry().smoke()
    assert "smoke: ok" in capsys.readouterr().out


def test_cli_info_and_help(capsys):
    from hola_amd.__main__ import main

    assert main(["info"]) == 0
    out = capsys.readouterr().out
    assert "physical cores" in out and "plan x8" in out
    assert main([]) == 0
