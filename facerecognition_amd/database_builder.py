"""Drop-in for the reference's ``inference/database_builder.py``: background build jobs that turn an
identity-per-folder image tree into an embeddings database (``{name: [512] f32}`` .npy).

Same classes and job protocol as the reference (BuildJob :19-87, DatabaseBuilder :89-234,
get_builder :241-243): status pending → running → completed | failed, progress 0-100, the last 50
log lines in ``to_dict()``, failures recorded with the traceback.  The ArcFace / FaceNet builders call
``extract_embeddings.build_db``, which embeds each identity's images in ONE batched ``fr_embed`` on
the GPU instead of one forward per image.

Differences, by design:
  * ``config["device"]`` defaults to ``"cuda"`` (the reference defaults to ``"cpu"``,
    database_builder.py:197,224); this package has no CPU compute path.
  * ``model_type == "lbph"`` (OpenCV LBPH training, :141-182) is outside the embedding hot path and
    fails the job with a clear message (out of scope).
"""
from __future__ import annotations

import threading
import traceback
from datetime import datetime
from typing import Callable, Dict, Optional


class BuildJob:
    def __init__(self, job_id: str, model_type: str, config: Dict):
        self.job_id = job_id
        self.model_type = model_type
        self.config = config
        self.status = "pending"
        self.progress = 0.0
        self.message = "Đang khởi tạo..."
        self.logs = []
        self.output_files = {}
        self.error = None
        self.start_time = None
        self.end_time = None

    def add_log(self, message: str):
        entry = f"[{datetime.now():%H:%M:%S}] {message}"
        self.logs.append(entry)
        print(entry)

    def update_progress(self, progress: float, message: str = None):
        self.progress = min(100.0, max(0.0, progress))
        if message:
            self.message = message
            self.add_log(message)

    def set_status(self, status: str):
        self.status = status
        if status == "running":
            self.start_time = datetime.now()
        elif status in ("completed", "failed"):
            self.end_time = datetime.now()

    def set_error(self, error: str):
        self.error = error
        self.add_log(f"ERROR: {error}")

    def add_output_file(self, label: str, path: str):
        self.output_files[label] = path
        self.add_log(f"Created: {label} -> {path}")

    def _get_elapsed_time(self) -> Optional[float]:
        if not self.start_time:
            return None
        return ((self.end_time or datetime.now()) - self.start_time).total_seconds()

    def to_dict(self) -> Dict:
        return {"job_id": self.job_id, "model_type": self.model_type, "status": self.status,
                "progress": self.progress, "message": self.message, "logs": self.logs[-50:],
                "output_files": self.output_files, "error": self.error,
                "elapsed_time": self._get_elapsed_time()}


DEFAULT_OUTPUT = {"arcface": "data/arcface_embeddings_db.npy", "facenet": "data/facenet_embeddings_db.npy"}
OUTPUT_LABEL = {"arcface": "ArcFace Database", "facenet": "FaceNet Database"}


class DatabaseBuilder:
    def __init__(self, build_fn: Callable = None):
        self.jobs: Dict[str, BuildJob] = {}
        self.lock = threading.Lock()
        self._build_fn = build_fn  # injectable for host-logic tests; default extract_embeddings.build_db

    def create_job(self, job_id: str, model_type: str, config: Dict) -> BuildJob:
        with self.lock:
            job = BuildJob(job_id, model_type, config)
            self.jobs[job_id] = job
            return job

    def get_job(self, job_id: str) -> Optional[BuildJob]:
        with self.lock:
            return self.jobs.get(job_id)

    def start_build(self, job_id: str) -> threading.Thread:
        job = self.get_job(job_id)
        if not job:
            raise ValueError(f"Job {job_id} không tồn tại")
        t = threading.Thread(target=self._run_build, args=(job,), daemon=True)
        t.start()
        return t

    def _run_build(self, job: BuildJob):
        try:
            job.set_status("running")
            job.update_progress(5, "Đang khởi tạo build process...")
            if job.model_type == "lbph":
                raise NotImplementedError("LBPH training is out of scope for facerecognition_amd "
                                          "(OpenCV LBPH, not on the embedding hot path)")
            if job.model_type not in ("arcface", "facenet"):
                raise ValueError(f"Model type không hợp lệ: {job.model_type}")
            self._build_embeddings(job)
            job.update_progress(100, "Hoàn thành!")
            job.set_status("completed")
        except Exception as e:  # reference :135-138
            job.set_error(str(e))
            job.add_log(traceback.format_exc())
            job.set_status("failed")

    def _build_embeddings(self, job: BuildJob):
        mt = job.model_type
        build = self._build_fn
        if build is None:
            from .extract_embeddings import build_db as build
        cfg = job.config
        job.update_progress(10, f"Đang load {'ArcFace' if mt == 'arcface' else 'FaceNet'} model...")
        save_path = cfg.get("output_path", DEFAULT_OUTPUT[mt])
        job.update_progress(20, f"Đang extract embeddings từ {cfg.get('data_dir')}...")
        build(model_path=cfg.get("model_path"), root_folder=cfg.get("data_dir"), save_path=save_path,
              device=cfg.get("device", "cuda"), use_face_detection=cfg.get("use_face_detection", True),
              model_type=mt)
        job.add_output_file(OUTPUT_LABEL[mt], save_path)


_builder = DatabaseBuilder()


def get_builder() -> DatabaseBuilder:
    return _builder
