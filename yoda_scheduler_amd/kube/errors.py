"""Kubernetes API errors (status codes the scheduler reacts to)."""
from __future__ import annotations


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str = "") -> None:
        super().__init__(f"{code} {reason}: {message}")
        self.code = code
        self.reason = reason
        self.message = message

    def status_obj(self) -> dict:
        return {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": self.message,
                "reason": self.reason, "code": self.code}


def not_found(what: str) -> ApiError:
    return ApiError(404, "NotFound", f"{what} not found")


def conflict(msg: str) -> ApiError:
    return ApiError(409, "Conflict", msg)


def already_exists(what: str) -> ApiError:
    return ApiError(409, "AlreadyExists", f"{what} already exists")


def gone(msg: str = "too old resource version") -> ApiError:
    return ApiError(410, "Expired", msg)


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.code == 409


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.code == 404
