"""Request batching engine + HTTP front end for the serving path (SURVEY §2.4 W8 taken to a service).

``BatchingEngine`` owns one model on one device: callers ``submit`` token-id prompts from any thread
and get a ``Future``; a single worker thread drains the queue every ``window_ms``, groups requests that
can share one static batch (same prompt length, new-token budget and sampling settings, up to
``max_batch``), and runs :func:`~.generate.generate` once per group — the decode steps of a whole group
then cost one HIP-graph replay each (``graph=True`` on a GPU).  One worker = one stream of GPU work, so
the model never runs concurrently with itself.

``create_app(engine)`` exposes it over HTTP (FastAPI): ``POST /generate`` with
``{"prompt": [ids], "max_new_tokens": n, "temperature": t, "top_k": k}`` returns
``{"tokens": [new ids], "batch": size of the batch it ran in}``; ``GET /health``.

    engine = BatchingEngine(model, max_batch=32)
    uvicorn.run(create_app(engine), host="0.0.0.0", port=8000)
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Tuple

import torch

from .generate import generate


class BatchingEngine:
    def __init__(self, model, max_batch: int = 32, window_ms: float = 5.0, graph: Optional[bool] = None,
                 device: Optional[torch.device] = None):
        self.model = model
        self.max_batch = max_batch
        self.window = window_ms / 1e3
        self.device = device or next(model.parameters()).device
        self.graph = (self.device.type == "cuda") if graph is None else graph
        self.q: "queue.Queue[Tuple[tuple, List[int], Future]]" = queue.Queue()
        self.batches_run = 0
        self._stop = threading.Event()
        self._lock = threading.Lock()  # submit's closed-check + enqueue vs close()
        self._thread = threading.Thread(target=self._loop, name="pda-serving", daemon=True)
        self._thread.start()

    def submit(self, prompt: List[int], max_new_tokens: int = 16, temperature: float = 0.0,
               top_k: Optional[int] = None) -> Future:
        if not prompt:
            raise ValueError("empty prompt")
        fut: Future = Future()
        with self._lock:
            if self._stop.is_set():
                raise RuntimeError("engine closed")
            self.q.put(((len(prompt), int(max_new_tokens), float(temperature), top_k), list(prompt), fut))
        return fut

    def close(self):
        """Stop the worker; every request not yet served fails with ``RuntimeError('engine closed')``
        instead of leaving its caller blocked."""
        with self._lock:
            self._stop.set()
        self._thread.join(timeout=10)
        self._fail_queued()

    def _fail_queued(self, pending=()):
        err = RuntimeError("engine closed")
        for _, _, fut in pending:
            if not fut.done():
                fut.set_exception(err)
        while True:
            try:
                _, _, fut = self.q.get_nowait()
            except queue.Empty:
                break
            if not fut.done():
                fut.set_exception(err)

    def _loop(self):
        # the current HIP device is per thread: make this worker's match the engine's device, or a
        # graph captured here would record on device 0's stream while the kernels run on cuda:N
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        pending: List[Tuple[tuple, List[int], Future]] = []
        try:
            self._serve(pending)
        finally:
            self._fail_queued(pending)

    def _serve(self, pending):
        while not self._stop.is_set():
            try:
                pending.append(self.q.get(timeout=0.05))
            except queue.Empty:
                if not pending:
                    continue
            deadline = time.monotonic() + self.window
            while time.monotonic() < deadline:
                try:
                    pending.append(self.q.get(timeout=max(0.0, deadline - time.monotonic())))
                except queue.Empty:
                    break
            groups: Dict[tuple, List[Tuple[List[int], Future]]] = {}
            for key, prompt, fut in pending:
                groups.setdefault(key, []).append((prompt, fut))
            pending.clear()
            for (T, new, temp, top_k), reqs in groups.items():
                for i in range(0, len(reqs), self.max_batch):
                    self._run(reqs[i: i + self.max_batch], new, temp, top_k)

    def _run(self, reqs, new, temp, top_k):
        try:
            prompt = torch.tensor([p for p, _ in reqs], dtype=torch.long, device=self.device)
            out = generate(self.model, prompt, new, temperature=temp, top_k=top_k,
                           graph=self.graph and new > 1)
            out = out[:, prompt.shape[1]:].cpu().tolist()
            self.batches_run += 1
            for (_, fut), toks in zip(reqs, out):
                fut.set_result({"tokens": toks, "batch": len(reqs)})
        except Exception as e:  # noqa: BLE001 - report to every waiting caller
            for _, fut in reqs:
                if not fut.done():
                    fut.set_exception(e)


def create_app(engine: BatchingEngine):
    from fastapi import FastAPI, HTTPException
    from pydantic import create_model

    # built at run time (this module uses postponed annotations, which FastAPI cannot resolve for
    # function-local models)
    GenerateRequest = create_model("GenerateRequest", prompt=(List[int], ...), max_new_tokens=(int, 16),
                                   temperature=(float, 0.0), top_k=(Optional[int], None))
    app = FastAPI(title="pytorchdistributed_amd serving")

    def health():
        return {"status": "ok", "device": str(engine.device), "batches_run": engine.batches_run}

    def gen(req):
        try:
            fut = engine.submit(req.prompt, req.max_new_tokens, req.temperature, req.top_k)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        except RuntimeError as e:  # engine closed
            raise HTTPException(status_code=503, detail=str(e))
        try:
            return fut.result(timeout=600)
        except RuntimeError as e:
            raise HTTPException(status_code=503, detail=str(e))

    gen.__annotations__ = {"req": GenerateRequest}
    app.get("/health")(health)
    app.post("/generate")(gen)
    return app
