"""Mirror of reference test/test_common.jl (Init / rank / size / printing / Finalize)."""
import pytest


def worker():
    import fluxmpi_amd as FluxMPI

    assert not FluxMPI.Initialized()
    try:
        FluxMPI.local_rank()
        raise AssertionError("local_rank before Init must raise")
    except FluxMPI.FluxMPINotInitializedError as e:
        assert "FluxMPI.init" in str(e)
    FluxMPI.Init(verbose=True)
    assert FluxMPI.Initialized()
    assert FluxMPI.local_rank() < FluxMPI.total_workers()
    assert FluxMPI.total_workers() >= 2
    FluxMPI.fluxmpi_println("Printing from Rank ", FluxMPI.local_rank())
    FluxMPI.fluxmpi_print("Printing from Rank ", FluxMPI.local_rank(), "\n")
    FluxMPI.Init(verbose=True)  # idempotent: "already initialized; Skipping..."
    FluxMPI.Finalize()
    assert FluxMPI.Finalized()
    assert FluxMPI.Initialized()  # reference: the flag is never reset


def test_common(spmd):
    spmd("tests.test_common:worker")


def test_single_process_world(capsys):
    """world == 1 path without a launcher (no process group needed)."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.parallel import runtime

    FluxMPI.fluxmpi_println("before init")  # prints a timestamp prefix, no error
    out = capsys.readouterr().out
    assert "before init" in out and out[:4].isdigit()
    if not runtime.Initialized():
        with pytest.warns(UserWarning, match="only 1 worker"):
            FluxMPI.Init(verbose=True, backend="gloo")
    assert FluxMPI.total_workers() == 1 and FluxMPI.local_rank() == 0
    FluxMPI.fluxmpi_println("hello ", 1)
    assert capsys.readouterr().out.endswith("hello 1\n")


def test_kernel_choice_table_roundtrip(tmp_path):
    """The shipped per-shape kernel-choice table (tuning/kernel_choices) loads into the autotune
    dictionaries and dumps back to the same records."""
    import json
    import os
    from fluxmpi_amd.ops import conv_choice as fb
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tuning", "kernel_choices", "resnet50_bs256.jsonl")
    saved = {name: dict(getattr(fb, name)) for name in fb._CHOICE_TABLES.values()}
    try:
        for name in fb._CHOICE_TABLES.values():
            getattr(fb, name).clear()
        n = fb.load_choices(path)
        assert n == sum(1 for line in open(path) if line.strip())
        assert fb._WG_CHOICE[("1x1", (256, 512, 28, 28), 256)] == ("w256", None)
        assert fb._FWD_ENGINE[((256, 64, 56, 56), 64)] == 7
        out = tmp_path / "c.jsonl"
        out.write_text("\n".join(fb.dump_choices()) + "\n")
        want = sorted(json.dumps(json.loads(line), sort_keys=True) for line in open(path) if line.strip())
        got = sorted(json.dumps(json.loads(line), sort_keys=True) for line in open(out) if line.strip())
        assert got == want
    finally:
        for name, d in saved.items():
            getattr(fb, name).clear()
            getattr(fb, name).update(d)


def test_kernel_choice_w3n_record_roundtrip():
    """A weight-gradient choice of the narrow 3x3 kernel (name + (variant, target workgroups))
    survives dump_choices / load_choice_lines — the form rank 0's table is broadcast in."""
    from fluxmpi_amd.ops import conv_choice as fb
    key = ("3x3", (256, 64, 56, 56), 64)
    saved = dict(fb._WG_CHOICE)
    try:
        fb._WG_CHOICE.clear()
        fb._WG_CHOICE[key] = ("w3n", (1, 256))
        lines = fb.dump_choices()
        fb._WG_CHOICE.clear()
        assert fb.load_choice_lines(lines) == 1
        assert fb._WG_CHOICE[key] == ("w3n", (1, 256))
        assert fb.w3n_configs(128) != fb.w3n_configs(64)
    finally:
        fb._WG_CHOICE.clear()
        fb._WG_CHOICE.update(saved)
