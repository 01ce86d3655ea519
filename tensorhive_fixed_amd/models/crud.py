"""CRUD mixin + serialisation contract shared by every ORM entity.

Reference: ``models/CRUDModel.py:11-94``.  ``save()`` runs ``check_assertions()`` then commits
(rollback + re-raise on SQLAlchemyError; AssertionError propagates); ``as_dict()`` camel-cases
the ``__public__`` (+ ``__private__``) attribute names and renders datetimes as
``YYYY-MM-DDTHH:MM:SS+00:00`` -- the web UI depends on both.
"""
from __future__ import annotations

import datetime
import logging
import re

from sqlalchemy.exc import MultipleResultsFound, NoResultFound, SQLAlchemyError

from ..database import db_session
from ..utils import dates

log = logging.getLogger(__name__)

_CAMEL = re.compile(r"_([a-z0-9])")


def camelcase(name: str) -> str:
    name = name.lstrip("_")
    return _CAMEL.sub(lambda m: m.group(1).upper(), name)


class CRUDModel:
    __public__: list[str] = ["id"]
    __private__: list[str] = []

    def check_assertions(self) -> None:  # pragma: no cover - overridden
        pass

    def save(self):
        try:
            self.check_assertions()
            db_session.add(self)
            db_session.commit()
        except SQLAlchemyError:
            db_session.rollback()
            log.error("saving %r failed", self)
            raise
        return self

    def destroy(self):
        try:
            db_session.delete(self)
            db_session.commit()
        except SQLAlchemyError:
            db_session.rollback()
            raise
        return self

    @classmethod
    def get(cls, id):
        try:
            return db_session.query(cls).filter_by(id=id).one()
        except MultipleResultsFound as e:
            raise MultipleResultsFound(f"multiple {cls.__name__} records with id={id}") from e
        except NoResultFound as e:
            raise NoResultFound(f"There is no record {cls.__name__} with id={id}!") from e

    @classmethod
    def all(cls):
        return db_session.query(cls).all()

    @staticmethod
    def _serialize(value):
        if isinstance(value, datetime.datetime):
            return dates.stringify(value)
        return value

    def as_dict(self, include_private: bool = False) -> dict:
        attrs = list(getattr(self, "__public__", ["id"]))
        if include_private:
            attrs += list(getattr(self, "__private__", []))
        return {camelcase(a): self._serialize(getattr(self, a)) for a in attrs}
