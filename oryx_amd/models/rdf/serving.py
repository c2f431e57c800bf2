"""RDF serving model and manager.

Equivalent of ``RDFServingModel`` (``[serving-app]/rdf/model/RDFServingModel.java:34-94``) and
``RDFServingModelManager.consume`` (``RDFServingModelManager.java:68-121``): ``predict``
returns the most probable class value or the numeric score (``Double.toString``); ``UP``
messages update a leaf found by ID in place (class counts, or running mean + count).
"""

from __future__ import annotations

import logging
from typing import Optional, Sequence

from ...api import AbstractServingModelManager, ServingModel
from ...utils import pmml as pmmlu, text
from ..classreg import CategoricalPrediction, NumericPrediction, data_to_example
from ..schema import InputSchema
from . import pmml as rdf_pmml

__all__ = ["RDFServingModel", "RDFServingModelManager"]

log = logging.getLogger(__name__)


class RDFServingModel(ServingModel):
    def __init__(self, forest, encodings, input_schema: InputSchema):
        if forest is None or encodings is None or input_schema is None:
            raise ValueError("forest, encodings and schema are required")
        self.forest = forest
        self.encodings = encodings
        self.input_schema = input_schema

    def predict(self, example: Sequence[str]) -> str:
        prediction = self.make_prediction(example)
        s = self.input_schema
        if s.is_classification():
            names = self.encodings.get_encoding_value_map(s.get_target_feature_index())
            return names[prediction.get_most_probable_category_encoding()]
        return text.java_double_str(prediction.get_prediction())

    def make_prediction(self, example: Sequence[str]):
        if len(example) != self.input_schema.get_num_features():
            raise ValueError("Wrong number of features")
        return self.forest.predict(data_to_example(example, self.input_schema, self.encodings))

    def get_forest(self):
        return self.forest

    def get_encodings(self):
        return self.encodings

    def get_input_schema(self) -> InputSchema:
        return self.input_schema

    def get_fraction_loaded(self) -> float:
        return 1.0

    def __repr__(self):
        return "RDFServingModel[numTrees:%d]" % len(self.forest.get_trees())


class RDFServingModelManager(AbstractServingModelManager):
    def __init__(self, config):
        super().__init__(config)
        self.input_schema = InputSchema(config)
        self.model: Optional[RDFServingModel] = None

    def consume(self, updates, context=None) -> None:
        for km in updates:
            if km.key is None:
                raise ValueError("Bad message: %r" % (km,))
            if km.key == "UP":
                if self.model is None:
                    continue
                update = text.read_json(km.message)
                tree = self.model.forest.get_trees()[int(update[0])]
                node = tree.find_by_id(str(update[1]))
                pred = node.get_prediction()
                if self.input_schema.is_classification():
                    for enc, count in update[2].items():
                        pred.update(int(enc), int(count))
                else:
                    pred.update(float(update[2]), int(update[3]))
            elif km.key in ("MODEL", "MODEL-REF"):
                log.info("Loading new model")
                pmml = pmmlu.read_pmml_from_update_key_message(km.key, km.message)
                rdf_pmml.validate_pmml_vs_schema(pmml, self.input_schema)
                forest, encodings = rdf_pmml.read(pmml)
                self.model = RDFServingModel(forest, encodings, self.input_schema)
                log.info("New model: %s", self.model)
            else:
                raise ValueError("Bad message: %r" % (km,))

    def get_model(self) -> Optional[RDFServingModel]:
        return self.model
