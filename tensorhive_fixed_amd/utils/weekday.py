"""Weekday enum used by restriction schedules (1 = Monday ... 7 = Sunday)."""
from enum import Enum


class Weekday(Enum):
    Monday = 1
    Tuesday = 2
    Wednesday = 3
    Thursday = 4
    Friday = 5
    Saturday = 6
    Sunday = 7

    def to_str(self) -> str:
        return self.name
