"""TEXBIAS_DEFER (INTEGRATION.md "Switches"): deferral is automatic inside DataLoader workers, off in the
main process, forced by ``set_deferred``, and turned off in workers by TEXBIAS_DEFER=0."""
import torch

from texbias import deferred


def test_defer_switch(monkeypatch):
    deferred.set_deferred(None)
    assert deferred.active() is False  # main process
    monkeypatch.setattr(torch.utils.data, "get_worker_info", lambda: object())
    assert deferred.active() is True  # a worker
    monkeypatch.setenv("TEXBIAS_DEFER", "0")
    assert deferred.active() is False
    deferred.set_deferred(True)
    try:
        assert deferred.active() is True
    finally:
        deferred.set_deferred(None)
