"""AutoML for time series (Py/automl): feature transformer, model zoo, recipes,
local trial search engine (one trial per GPU when parallel), pipelines."""
