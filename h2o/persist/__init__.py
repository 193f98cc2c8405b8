"""``h2o.persist`` (reference: h2o-py/h2o/persist): S3 credentials of the object-store persist layer."""
from .. import remove_s3_credentials, set_s3_credentials

__all__ = ["set_s3_credentials", "remove_s3_credentials"]
