"""In-process stand-in for FEDn's combiner UpdateHandler (fedn/network/combiner/updatehandler.py).

Exposes exactly the surface the aggregator plug-ins consume:
``model_updates`` (a FIFO ``queue.Queue``), ``next_model_update()``,
``load_model_update(mu, helper) -> (arrays, training_metadata)``, ``load_model(helper,
model_id)`` and ``delete_model(mu)``. Models live in a dict instead of the combiner's
temp-file store + npz codec, so tests and benchmarks can drive the plug-ins without
gRPC. Behaviour mirrors updatehandler.py:35-117: metadata must carry
``training_metadata.num_examples`` (else the update is rejected at ingest, :72-88) and
``round_id`` is copied from the config (:106-116).
"""
import json
import os
import queue
import uuid
from dataclasses import dataclass
from io import BytesIO


class _NpzBytes:
    __slots__ = ("data",)

    def __init__(self, data):
        self.data = data


@dataclass
class ModelUpdate:
    """The fields of fedn.proto ``ModelUpdate`` (fedn.proto:67-76) the aggregators read."""

    model_id: str
    model_update_id: str
    meta: str
    config: str = "{}"


class MemoryModelStore:
    def __init__(self):
        self.models = {}

    def put(self, model_id, arrays):
        self.models[model_id] = arrays

    def get(self, model_id):
        return self.models.get(model_id)

    def delete(self, model_id):
        return self.models.pop(model_id, None) is not None


class TempFileModelStore:
    """FEDn's TempModelStorage (tempmodelstorage.py:11-76) as far as the round sees it: an update's
    bytes live in a file under ``directory`` (FEDN_MODEL_DIR), ``get`` reads the whole file back
    (:27-41), ``delete`` is ``os.remove`` (:66-76). Non-bytes models (global models as arrays, the
    tests' host updates) stay in memory. With MemoryModelService it is written chunk by chunk as
    ModelService.Upload writes it (get_ptr, :43-53)."""

    def __init__(self, directory=None):
        import tempfile
        self.dir = directory or tempfile.mkdtemp(prefix="fedn_models_")
        self.models = {}
        self._files = {}

    def path(self, model_id):
        return os.path.join(self.dir, str(model_id))

    def open_write(self, model_id):
        f = self._files.get(model_id)
        if f is None:
            f = self._files[model_id] = open(self.path(model_id), "wb")
        return f

    def commit(self, model_id):
        f = self._files.pop(model_id, None)
        if f is not None:
            f.close()
        self.models[model_id] = _ON_DISK

    def put(self, model_id, arrays):
        if isinstance(arrays, _NpzBytes):
            with open(self.path(model_id), "wb") as f:
                f.write(arrays.data)
            arrays = _ON_DISK
        self.models[model_id] = arrays

    def get(self, model_id):
        m = self.models.get(model_id)
        if m is _ON_DISK:
            with open(self.path(model_id), "rb") as f:
                return _NpzBytes(f.read())
        return m

    def delete(self, model_id):
        m = self.models.pop(model_id, None)
        if m is _ON_DISK:
            os.remove(self.path(model_id))
        return m is not None


_ON_DISK = object()

MODEL_STATUS_OK = 0            # fedn.proto:147-153 (ModelStatus)
MODEL_STATUS_IN_PROGRESS = 1
CHUNK_SIZE = 1 << 20           # modelservice.py:12


@dataclass
class ModelRequest:
    """The fields of fedn.proto ``ModelRequest`` that ModelService.Upload reads."""

    id: str
    data: bytes = b""
    status: int = MODEL_STATUS_IN_PROGRESS


@dataclass
class ModelResponse:
    id: str
    status: int
    message: str = ""


def upload_requests(data, model_id, chunk=CHUNK_SIZE):
    """The request stream a FEDn client sends (upload_request_generator, modelservice.py:15-31):
    ``chunk``-byte IN_PROGRESS requests, then an empty OK request."""
    mv = memoryview(data)
    for o in range(0, len(mv), chunk):
        yield ModelRequest(id=model_id, data=bytes(mv[o:o + chunk]), status=MODEL_STATUS_IN_PROGRESS)
    yield ModelRequest(id=model_id, data=b"", status=MODEL_STATUS_OK)


class MemoryModelService:
    """``ModelService.Upload`` (modelservice.py:198-221) over the in-memory store: chunks are
    kept per id; the OK request commits the bytes under that id and ends the call. FEDn writes
    each chunk to a temp file (a write that releases the GIL); the stand-in keeps the chunk
    objects and joins them once (a join of that size releases the GIL too) rather than growing
    one bytearray, whose reallocations copy the upload over and over under the GIL and starve
    the threads decoding other uploads."""

    def __init__(self, store):
        self.store = store
        self._parts = {}

    def Upload(self, request_iterator, context):
        to_file = isinstance(self.store, TempFileModelStore)
        for request in request_iterator:
            if request.status == MODEL_STATUS_IN_PROGRESS:
                if to_file:                     # modelservice.py:208-214: each chunk written to the file
                    self.store.open_write(request.id).write(request.data)
                else:
                    self._parts.setdefault(request.id, []).append(bytes(request.data))
            if request.status == MODEL_STATUS_OK and not request.data:
                if to_file:
                    self.store.commit(request.id)
                else:
                    self.store.put(request.id, _NpzBytes(b"".join(self._parts.pop(request.id, []))))
                return ModelResponse(id=request.id, status=MODEL_STATUS_OK, message="Got model successfully.")
        return None


class MemoryUpdateHandler:
    def __init__(self, store=None):
        self.model_updates = queue.Queue()
        self.store = store or MemoryModelStore()

    # --- producer side (what Combiner.SendModelUpdate -> on_model_update does) ----------
    def put_global_model(self, arrays, model_id=None):
        model_id = model_id or str(uuid.uuid4())
        self.store.put(model_id, arrays)
        return model_id

    def submit_bytes(self, npz_bytes, num_examples, model_id="global", round_id="1", via=None):
        """Enqueue an update held as npz bytes (what ModelService.Upload stores, modelservice.py:198-221)."""
        return self.submit(_NpzBytes(bytes(npz_bytes)), num_examples, model_id, round_id, via)

    def submit(self, arrays, num_examples, model_id="global", round_id="1", via=None):
        """Store an update and enqueue its ModelUpdate (on_model_update, updatehandler.py:46-70).
        ``via``: a wrapper (e.g. ingest.StagingUpdateHandler) whose on_model_update to call."""
        uid = str(uuid.uuid4())
        self.store.put(uid, arrays)
        meta = json.dumps({"training_metadata": {"num_examples": num_examples},
                           "config": json.dumps({"round_id": round_id})})
        mu = ModelUpdate(model_id=model_id, model_update_id=uid, meta=meta)
        (via or self).on_model_update(mu)
        return mu

    def submit_uploaded(self, model_update_id, num_examples, model_id="global", round_id="1", via=None):
        """Enqueue the ModelUpdate of an update already uploaded under ``model_update_id``
        (the client's Upload, then SendModelUpdate, combiner.py:783-797)."""
        meta = json.dumps({"training_metadata": {"num_examples": num_examples},
                           "config": json.dumps({"round_id": round_id})})
        mu = ModelUpdate(model_id=model_id, model_update_id=model_update_id, meta=meta)
        (via or self).on_model_update(mu)
        return mu

    def on_model_update(self, model_update):
        try:
            json.loads(model_update.meta)["training_metadata"]["num_examples"]
        except (KeyError, TypeError, ValueError):
            return False
        self.model_updates.put(model_update)
        return True

    # --- consumer side (what the aggregators call) -------------------------------------
    def next_model_update(self):
        return self.model_updates.get(block=False)

    def load_model(self, helper, model_id):
        model = self.store.get(model_id)
        if model is None:
            raise RuntimeError(f"Failed to load model {model_id}.")
        if isinstance(model, _NpzBytes):        # load_model_from_bytes(..., helper) (modelservice.py:110-125)
            if helper is None:
                raise RuntimeError("an npz-encoded update needs a helper to decode it")
            return helper.load(BytesIO(model.data))
        return model

    def load_model_update_byte(self, model_update):
        """(raw npz bytes, training_metadata) — updatehandler.py:119-144."""
        model = self.store.get(model_update.model_update_id)
        if not isinstance(model, _NpzBytes):
            raise RuntimeError("update is not held as bytes")
        metadata = json.loads(model_update.meta)
        config = json.loads(metadata["config"]) if "config" in metadata else json.loads(model_update.config)
        training_metadata = metadata["training_metadata"]
        if "round_id" in config:
            training_metadata["round_id"] = config["round_id"]
        return model.data, training_metadata

    def load_model_update(self, model_update, helper):
        model = self.load_model(helper, model_update.model_update_id)
        metadata = json.loads(model_update.meta)
        config = json.loads(metadata["config"]) if "config" in metadata else json.loads(model_update.config)
        training_metadata = metadata["training_metadata"]
        if "round_id" in config:
            training_metadata["round_id"] = config["round_id"]
        return model, training_metadata

    def delete_model(self, model_update):
        self.store.delete(model_update.model_update_id)
