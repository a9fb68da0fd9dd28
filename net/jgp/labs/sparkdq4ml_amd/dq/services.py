"""DQ business rules — scalar reference semantics.

* ``check_minimum_price`` == ``MinimumPriceDataQualityService.checkMinimumPrice``
  (``MinimumPriceDataQualityService.java:5-13``): ``price < 20 -> -1`` else ``price``.
* ``check_price_range`` == ``PriceCorrelationDataQualityService.checkPriceRange``
  (``PriceCorrelationDataQualityService.java:5-10``): ``guest < 14 && price > 90 -> -1`` else
  ``price``.

These scalar forms are what Java-style callers use; the vectorized/fused forms of the same rules
are the IR builders in :mod:`.rules`.
"""
from __future__ import annotations

MIN_PRICE = 20
CORRELATION_MAX_GUESTS = 14
CORRELATION_MAX_PRICE = 90


def check_minimum_price(price: float) -> float:
    if price < MIN_PRICE:
        return -1.0
    return float(price)


def check_price_range(price: float, guest: int) -> float:
    if guest < CORRELATION_MAX_GUESTS and price > CORRELATION_MAX_PRICE:
        return -1.0
    return float(price)


# Java spellings
checkMinimumPrice = check_minimum_price
checkPriceRange = check_price_range
