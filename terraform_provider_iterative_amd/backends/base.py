"""Task interface (reference: ``task/task.go:48-67`` and ``task/common/resource.go``)."""
from __future__ import annotations

import abc
from typing import Dict, List

from ..models.values import Event
from ..utils.identifier import Identifier


class Resource(abc.ABC):
    """``common.Resource``: every cloud object has Read/Create/Delete."""

    @abc.abstractmethod
    def read(self) -> None: ...

    @abc.abstractmethod
    def create(self) -> None: ...

    @abc.abstractmethod
    def delete(self) -> None: ...


class Task(Resource):
    @abc.abstractmethod
    def start(self) -> None: ...

    @abc.abstractmethod
    def stop(self) -> None: ...

    @abc.abstractmethod
    def push(self) -> None:
        """Upload the task's workdir to its storage."""

    @abc.abstractmethod
    def pull(self) -> None:
        """Download the output directory from storage."""

    @abc.abstractmethod
    def status(self) -> Dict[str, int]: ...

    @abc.abstractmethod
    def events(self) -> List[Event]: ...

    @abc.abstractmethod
    def logs(self) -> List[str]: ...

    @abc.abstractmethod
    def get_identifier(self) -> Identifier: ...

    @abc.abstractmethod
    def get_addresses(self) -> List[str]: ...

    @abc.abstractmethod
    def get_key_pair(self):
        """Deterministic SSH key pair, or raise ``NotImplementedErr``."""
