"""dq4ml — an MI355X-native data-quality + machine-learning tabular pipeline engine with the
Spark API surface of the ``net.jgp.labs.sparkdq4ml`` lab.

    from net.jgp.labs.sparkdq4ml_amd import SparkSession, callUDF, VectorAssembler, LinearRegression
"""
from .sql.session import SparkSession
from .sql.dataframe import DataFrame, Row
from .sql.column import Column
from .sql.functions import callUDF, call_udf, col, lit, udf, when, expr, coalesce
from .sql.types import DataTypes, StructType, StructField
from .models.linalg import Vectors, DenseVector, SparseVector, Vector
from .models.feature import VectorAssembler
from .models.regression import (LinearRegression, LinearRegressionModel,
                                LinearRegressionTrainingSummary)
from .dq.rules import MinimumPriceDataQualityUdf, PriceCorrelationDataQualityUdf

__version__ = "0.1.0"

__all__ = [
    "SparkSession", "DataFrame", "Row", "Column", "callUDF", "call_udf", "col", "lit", "udf", "when",
    "expr", "coalesce", "DataTypes", "StructType", "StructField", "Vectors", "DenseVector",
    "SparseVector", "Vector", "VectorAssembler", "LinearRegression", "LinearRegressionModel",
    "LinearRegressionTrainingSummary", "MinimumPriceDataQualityUdf", "PriceCorrelationDataQualityUdf",
]
